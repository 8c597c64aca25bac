"""The native apps (csrc/apps, reference bin/*.cu) on one MI355X: each runs a small case on the device backend and
prints the reference's CSV line (formats pinned on the CPU path in test_apps.py). Covers the apps whose reference
versions are GPU-only (bench_alltoallv, measure_buf_exchange, the device pingpong)."""
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "build", "bin")
NUM = r"[-+0-9.e]+"

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not os.path.exists(os.path.join(BIN, "jacobi3d")), reason="native apps not built")]


def run_app(*argv, timeout=100):
    env = dict(os.environ)
    env["STENCIL_PLAN_FILE"] = "0"
    for k in ("RANK", "WORLD_SIZE", "STENCIL_RANK", "STENCIL_WORLD_SIZE"):
        env.pop(k, None)
    p = subprocess.run([os.path.join(BIN, argv[0]), *map(str, argv[1:])], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=timeout, cwd="/tmp")
    assert p.returncode == 0, p.stdout[-3000:]
    return p.stdout


@pytest.mark.parametrize("temporal", [1, 2])
def test_jacobi3d_device(temporal):
    out = run_app("jacobi3d", 128, 128, 128, "-n", 4, "--temporal", temporal)
    m = re.search(rf"^jacobi3d,([a-z/]+),1,\d+,128,128,128,({NUM}),({NUM}),({NUM})$", out, re.M)
    assert m, out[-2000:]
    assert float(m.group(4)) > 0


@pytest.mark.parametrize("temporal", [1, 2])
def test_jacobi3d_device_result_vs_oracle(tmp_path, temporal):
    """The jacobi3d app on the GPU: its final ParaView dump equals the torch oracle (warm-up + timed sweeps =
    4 x temporal steps; the dump prints 6 decimals)."""
    import torch

    from stencil2_amd.ops import jacobi_step_reference
    from stencil2_amd.utils.paraview import paraview_grid

    n = 48
    run_app("jacobi3d", n, n, n, "-n", 3, "--warmup", 1, "--temporal", temporal, "--paraview", "--prefix",
            str(tmp_path) + "/")
    got = paraview_grid(str(tmp_path / "jacobi3d_final"), "d", (n, n, n))
    u = torch.full((n, n, n), 0.5, dtype=torch.float32)
    for _ in range(4 * temporal):
        u = jacobi_step_reference(u)
    assert (got - u.double()).abs().max().item() <= 5.01e-7


def test_astaroth_sim_device():
    out = run_app("astaroth_sim", "--x", 96, "--y", 96, "--z", 96, "--q", 2, "-n", 2)
    assert re.search(rf"^astaroth,[a-z/]+,1,96,96,96,2,{NUM},{NUM},{NUM},{NUM}$", out, re.M), out[-2000:]


def test_bench_exchange_device():
    out = run_app("bench_exchange", "--x", 64, "--y", 64, "--z", 64, "--fr", 2, "--iters", 3)
    rows = re.findall(rf"^64-64-64/([a-z&]+)/[0-9/]+,3,({NUM}),({NUM}),{NUM},{NUM},{NUM},{NUM}$", out, re.M)
    assert {"faces", "uniform"} <= {r[0] for r in rows}, out[-2000:]
    assert all(float(r[2]) > 0 for r in rows)


def test_weak_and_weak_exchange_device():
    out = run_app("weak", 64, 64, 64, 2)
    assert re.search(r"^weak,[a-z/]+,64,64,64,262144,", out, re.M), out[-2000:]
    out = run_app("weak_exchange", 64, 64, 64, 2)
    assert re.search(rf"^weak_exchange,[a-z/]+,1,64,64,64,2,{NUM},{NUM}$", out, re.M), out[-2000:]


@pytest.mark.parametrize("flags", [["--x-face-lines"], ["--x-face-lines-auto", 0], ["--interior-align", 64]])
def test_exchange_apps_layout_flags_device(flags):
    """The layout / x-face flags on the device path (astaroth_sim --no-wrap exchanges every halo each step)."""
    out = run_app("astaroth_sim", "--x", 96, "--y", 96, "--z", 96, "--q", 2, "-n", 2, "--no-wrap", *flags)
    assert re.search(rf"^astaroth,[a-z/]+,1,96,96,96,2,{NUM},{NUM},{NUM},{NUM}$", out, re.M), out[-2000:]
    out = run_app("bench_exchange", "--x", 64, "--y", 64, "--z", 64, "--fr", 2, "--iters", 3, *flags)
    assert re.search(r"^64-64-64/faces/2,3,", out, re.M), out[-2000:]


def test_bench_pack_device():
    out = run_app("bench_pack", "--n", 64, "--iters", 2)
    assert re.search(rf"^64,\[0;0;1\],{NUM},{NUM},{NUM},{NUM},{NUM}$", out, re.M), out[-2000:]


def test_bench_alltoallv_and_measure_buf_exchange():
    out = run_app("bench_alltoallv", "--iters", 2)
    assert out.startswith("name,gpus,total_bytes,seconds,GBps"), out[-2000:]
    assert re.findall(r"^[a-zA-Z0-9_+-]+,1,\d+,", out, re.M), out[-2000:]
    out = run_app("measure_buf_exchange", "--rounds", 2, "--target-ms", 0.5)
    assert re.search(r"^round \d+: 0>0 [0-9.]+ms/[0-9.]+MiB", out, re.M), out[-2000:]


def test_bench_py_json_contract():
    """bench.py on one GPU prints one JSON line with the driver's fields (exact 512^3 grid, fused triples)."""
    import json
    import sys
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "4", "--warmup", "2",
                        "--exchange-iters", "2"], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=100, cwd=REPO)
    assert p.returncode == 0, p.stdout[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-3000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["warmup"] == 2 and d["value"] > 0
    assert d["config"]["grid"] == [512, 512, 512] and d["config"]["temporal"] == 3
