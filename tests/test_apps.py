"""The native apps (csrc/apps, reference bin/*.cu) on the CPU path: each runs on a tiny grid through the host
backend (no GPU in the process) and prints the reference's CSV line. Multi-rank apps run as ranks of the native TCP
process group (the reference's mpirun). These pin the CLI and output formats the reference's scripts parse."""
import os
import re
import subprocess

import pytest

from conftest import free_port

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "build", "bin")
NUM = r"[-+0-9.e]+"

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(BIN, "jacobi3d")),
                                reason="native apps not built (python -c 'import __graft_entry__ as g; g.build()')")


def _env():
    env = dict(os.environ)
    env.update({"STENCIL_PLAN_FILE": "0", "OMP_NUM_THREADS": "1", "HIP_VISIBLE_DEVICES": "",
                "ROCR_VISIBLE_DEVICES": ""})
    for k in ("RANK", "WORLD_SIZE", "STENCIL_RANK", "STENCIL_WORLD_SIZE"):
        env.pop(k, None)
    return env


def run_app(*argv, timeout=120):
    p = subprocess.run([os.path.join(BIN, argv[0]), *map(str, argv[1:])], env=_env(), stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=timeout, cwd="/tmp")
    assert p.returncode == 0, p.stdout[-3000:]
    return p.stdout


def run_app_ranks(n, *argv, timeout=120):
    """`n` ranks of one native TCP process group; returns [(rc, output)] per rank."""
    port = free_port()
    procs = []
    for r in range(n):
        env = _env()
        env.update({"STENCIL_RANK": str(r), "STENCIL_WORLD_SIZE": str(n), "STENCIL_MASTER_ADDR": "127.0.0.1",
                    "STENCIL_MASTER_PORT": str(port)})
        procs.append(subprocess.Popen([os.path.join(BIN, argv[0]), *map(str, argv[1:])], env=env, cwd="/tmp",
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, out))
    return outs


def test_jacobi3d_csv():
    """bin/jacobi3d.cu:339-341: jacobi3d,<methods>,<ranks>,<devCount>,x,y,z,<min s>,<trimean s> (+ Gcells/s)."""
    out = run_app("jacobi3d", 16, 16, 16, "-n", 2)
    m = re.search(rf"^jacobi3d,([a-z/]+),1,0,16,16,16,({NUM}),({NUM}),({NUM})$", out, re.M)
    assert m, out[-2000:]
    assert float(m.group(2)) > 0 and float(m.group(4)) > 0


def _check_jacobi_dump(prefix, n, steps):
    """The app's final ParaView dump vs the torch oracle after `steps` steps from the 0.5 initial field (the dump
    prints 6 decimals: |err| <= 5e-7)."""
    import torch

    from stencil2_amd.ops import jacobi_step_reference
    from stencil2_amd.utils.paraview import paraview_grid

    got = paraview_grid(prefix, "d", (n, n, n))
    u = torch.full((n, n, n), 0.5, dtype=torch.float32)
    for _ in range(steps):
        u = jacobi_step_reference(u)
    err = (got - u.double()).abs().max().item()
    assert err <= 5.01e-7, err


@pytest.mark.parametrize("temporal", [1, 2])
def test_jacobi3d_result_vs_oracle(tmp_path, temporal):
    """The jacobi3d app's field (its final ParaView dump) equals the torch oracle, not just its CSV shape:
    host backend (no fused pairs there: --temporal 2 runs single steps), warm-up + timed sweeps = 4 steps."""
    n = 24
    run_app("jacobi3d", n, n, n, "-n", 3, "--warmup", 1, "--temporal", temporal, "--paraview", "--prefix",
            str(tmp_path) + "/")
    _check_jacobi_dump(str(tmp_path / "jacobi3d_final"), n, 4)


def test_jacobi3d_two_ranks_weak_scaled():
    """Two ranks: the global grid follows the reference weak-scaling rule (24 * 2^0.33333 -> 30), rank 0 prints."""
    outs = run_app_ranks(2, "jacobi3d", 24, 24, 24, "-n", 2)
    for rc, out in outs:
        assert rc == 0, out[-3000:]
    assert re.search(rf"^jacobi3d,[a-z/]+,2,0,30,30,30,{NUM},{NUM},{NUM}$", outs[0][1], re.M), outs[0][1][-2000:]


def test_astaroth_sim_csv():
    out = run_app("astaroth_sim", "--x", 16, "--y", 16, "--z", 16, "--q", 2, "-n", 2)
    assert re.search(rf"^astaroth,[a-z/]+,1,16,16,16,2,{NUM},{NUM},{NUM},{NUM}$", out, re.M), out[-2000:]


def test_bench_exchange_csv():
    """bin/bench_exchange.cu: one row per radius pattern, name,count,trimean (S),trimean (B/s),stddev,min,avg,max."""
    out = run_app("bench_exchange", "--x", 16, "--y", 16, "--z", 16, "--fr", 1, "--iters", 3)
    rows = re.findall(rf"^16-16-16/([a-z&]+)/[0-9/]+,3,({NUM}),({NUM}),{NUM},{NUM},{NUM},{NUM}$", out, re.M)
    names = {r[0] for r in rows}
    assert {"faces", "fec", "uniform"} <= names, out[-2000:]
    assert all(float(r[1]) > 0 and float(r[2]) > 0 for r in rows)


def test_weak_and_weak_exchange_csv():
    out = run_app("weak", 16, 16, 16, 2)
    assert re.search(r"^weak,[a-z/]+,16,16,16,4096,", out, re.M), out[-2000:]
    out = run_app("weak_exchange", 16, 16, 16, 2)
    assert re.search(rf"^weak_exchange,[a-z/]+,1,16,16,16,2,{NUM},{NUM}$", out, re.M), out[-2000:]


def test_layout_and_x_face_flags_on_every_exchange_app():
    """--interior-align, --x-face-lines and --x-face-lines-auto (app::MethodArgs) are accepted by every exchange
    app; a bad alignment is refused with the LocalDomain message."""
    flags = ["--interior-align", 64, "--x-face-lines", "--x-face-lines-auto", 0]
    run_app("weak", 16, 16, 16, 2, *flags)
    run_app("weak_exchange", 16, 16, 16, 2, *flags)
    run_app("astaroth_sim", "--x", 16, "--y", 16, "--z", 16, "--q", 2, "-n", 2, "--no-wrap", *flags)
    run_app("bench_exchange", "--x", 16, "--y", 16, "--z", 16, "--fr", 1, "--iters", 2, *flags)
    p = subprocess.run([os.path.join(BIN, "weak"), "16", "16", "16", "2", "--interior-align", "96"], env=_env(),
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=60, cwd="/tmp")
    assert p.returncode != 0 and "interior alignment must be 64 or 128" in p.stdout, p.stdout[-2000:]


def test_bench_qap_and_pack():
    out = run_app("bench_qap")
    for name in ("random", "matched", "blockdiag"):
        assert re.search(rf"^{name},\d+,", out, re.M), out[-2000:]
    out = run_app("bench_pack", "--n", 16, "--iters", 2)
    # one row per direction class: n,[dx;dy;dz],bytes,pack s,unpack s,pack GB/s,unpack GB/s
    assert re.search(rf"^16,\[0;0;1\],3072,{NUM},{NUM},{NUM},{NUM}$", out, re.M), out[-2000:]


def test_pingpong_host_two_ranks():
    outs = run_app_ranks(2, "pingpong", "--host", "--min", 4, "--max", 8, "--iters", 2)
    for rc, out in outs:
        assert rc == 0, out[-3000:]
    sizes = [int(m) for m in re.findall(rf"^tcp-host,(\d+),1,{NUM},{NUM}$", outs[0][1], re.M)]
    assert sizes == [16, 32, 64, 128, 256], outs[0][1][-2000:]
