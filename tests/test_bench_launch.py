"""bench.py --gpus N: one fresh rank per GPU spawned before torch is imported, failures stop every sibling, and a
--gpus / WORLD_SIZE mismatch is refused (reference scripts/summit/weak_256n.sh:26-30 launches one
rank per GPU). CPU only: STENCIL_BENCH_DRY makes each rank report its layout instead of running the bench."""
import json
import os
import subprocess
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env["STENCIL_BENCH_DRY"] = "1"
    env.update(kw)
    return env


@pytest.mark.parametrize("n", [2, 3, 8])
def test_gpus_n_spawns_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--steps", "2"], env=_env(), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert sorted(l["rank"] for l in lines) == list(range(n))
    assert all(l["world"] == n and l["local_rank"] == l["rank"] for l in lines)
    assert len({l["master"] for l in lines}) == 1 and lines[0]["master"].startswith("127.0.0.1:")
    # the ranks are fresh interpreters: nothing imported torch (or initialised HIP) before the fork
    assert not any(l["torch_loaded"] for l in lines)


def test_failing_rank_stops_siblings():
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4"],
                       env=_env(STENCIL_BENCH_DRY_FAIL_RANK="2", STENCIL_BENCH_DRY_SLEEP="300"), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    assert time.monotonic() - t0 < 60, "siblings of the failed rank were not stopped"
    assert "rank 2 exited with 3" in r.stderr


def test_launch_timeout_stops_all():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--launch-timeout", "2"],
                       env=_env(STENCIL_BENCH_DRY_SLEEP="300"), capture_output=True, text=True, timeout=120)
    assert r.returncode == 124, r.stderr[-2000:]


def test_world_size_mismatch_is_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4"], env=_env(WORLD_SIZE="2", RANK="0"),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 2
    assert "--gpus 4 but WORLD_SIZE=2" in r.stderr


def test_world_size_match_under_launcher_runs_as_rank():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2"], env=_env(WORLD_SIZE="2", RANK="1", LOCAL_RANK="1"),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]
    assert json.loads(r.stdout.strip())["rank"] == 1


def test_launch_module_native_app_style():
    """python -m stencil2_amd.launch semantics via spawn_ranks: every rank sees its own STENCIL_RANK."""
    sys.path.insert(0, REPO)
    import importlib.util
    spec = importlib.util.spec_from_file_location("_l", os.path.join(REPO, "stencil2_amd", "launch.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    code = "import os,sys; sys.exit(0 if os.environ['STENCIL_RANK']==os.environ['RANK'] else 5)"
    assert m.spawn_ranks([sys.executable, "-c", code], 3, timeout=60) == 0
    assert m.spawn_ranks([sys.executable, "-c", "import sys; sys.exit(7)"], 2, timeout=60) == 7
