import os
import socket
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
os.environ.setdefault("STENCIL_PLAN_FILE", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def st():
    import stencil2_amd

    return stencil2_amd


def has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def run_ranks(n, script, args=(), env_extra=None, per_rank_env=None, timeout=240):
    """Launch `n` python processes running `script` as ranks of one native TCP process group."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"STENCIL_RANK": str(r), "STENCIL_WORLD_SIZE": str(n), "STENCIL_MASTER_ADDR": "127.0.0.1",
                    "STENCIL_MASTER_PORT": str(port), "PYTHONPATH": REPO, "STENCIL_SKIP_BUILD": "1",
                    "STENCIL_PLAN_FILE": "0", "OMP_NUM_THREADS": "1"})
        env.pop("RANK", None)
        env.pop("WORLD_SIZE", None)
        if env_extra:
            env.update(env_extra)
        if env.get("MP_DEVICE") == "1" and "GPU_MAX_HW_QUEUES" not in env:
            # ranks sharing the one GPU: at most 8 hardware queues in all, or the GPU time-slices the processes'
            # queues (bench.py _limit_queues_when_sharing, profiles/r3/cliff/)
            env["GPU_MAX_HW_QUEUES"] = str(max(1, 8 // n))
        if per_rank_env:
            env.update(per_rank_env(r))
        procs.append(subprocess.Popen([sys.executable, script, *map(str, args)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            # report where every rank was (its output so far) instead of a bare timeout
            for q in procs:
                q.kill()
            tails = []
            for r, q in enumerate(procs):
                try:
                    o, _ = q.communicate(timeout=10)
                except Exception:  # noqa: BLE001
                    o = "<no output>"
                tails.append(f"--- rank {r} (rc {q.returncode}) ---\n{(o or '')[-2000:]}")
            raise AssertionError(f"ranks timed out after {timeout} s\n" + "\n".join(tails))
        outs.append((p.returncode, out))
    return outs
