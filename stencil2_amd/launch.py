"""Launch N ranks of a native app or Python script on this node (an `mpirun -n` / `jsrun -a N` equivalent for the
TCP process group and torch.distributed): python -m stencil2_amd.launch -n 4 build/bin/jacobi3d 256 256 256 -n 20

The reference's sweeps start one rank per GPU from the job script (scripts/summit/weak_256n.sh:26-30, `jsrun -a 6
-g 6`); here `spawn_ranks` does it from Python. It is stdlib-only and never touches the GPU, so `bench.py --gpus N`
can load it by path (without importing torch or the package) and fork the ranks before any HIP call.

Failure handling: the parent polls every rank; the first rank that exits non-zero (or the overall timeout) kills
every sibling (SIGTERM, then SIGKILL after a grace period) instead of leaving them blocked in a collective until
their own transport timeout, and the parent exits with that rank's code (124 on timeout). Children also get
PR_SET_PDEATHSIG, so a parent killed outright takes its ranks with it.
"""
from __future__ import annotations

import argparse
import ctypes
import os
import signal
import socket
import subprocess
import sys
import time


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_env(rank: int, world: int, port: int, stencil_port: int, base: dict | None = None) -> dict:
    """torch.distributed (env://, MASTER_PORT) and native TCP-group (STENCIL_MASTER_PORT) rendezvous variables of
    one rank on this node."""
    env = dict(os.environ if base is None else base)
    env.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
               GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
               STENCIL_RANK=str(rank), STENCIL_WORLD_SIZE=str(world), STENCIL_MASTER_ADDR="127.0.0.1",
               STENCIL_MASTER_PORT=str(stencil_port))
    return env


def _die_with_parent():
    try:  # Linux: SIGKILL this child when the launching process dies
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, int(signal.SIGKILL))  # PR_SET_PDEATHSIG
    except OSError:
        pass


def _stop(procs, grace: float = 10.0):
    for p in procs:
        if p.poll() is None:
            try:
                p.terminate()
            except OSError:
                pass
    t0 = time.monotonic()
    for p in procs:
        try:
            p.wait(timeout=max(0.1, grace - (time.monotonic() - t0)))
        except subprocess.TimeoutExpired:
            pass
    for p in procs:
        if p.poll() is None:
            try:
                p.kill()
                p.wait(timeout=5)
            except (OSError, subprocess.TimeoutExpired):
                pass


def spawn_ranks(cmd: list[str], n: int, timeout: float | None = None, port: int | None = None,
                env_fn=None, poll_s: float = 0.1, log=sys.stderr) -> int:
    """Run `cmd` as ranks 0..n-1 (one process each, rendezvous on 127.0.0.1) and wait for all of them.

    Returns 0 when every rank exits 0; otherwise the first failing rank's exit code (a signal -s becomes 128+s), or
    124 when `timeout` seconds pass first. Any failure or the timeout stops every other rank."""
    port = free_port() if port is None else port
    stencil_port = free_port()
    while stencil_port == port:
        stencil_port = free_port()
    procs = []
    try:
        for r in range(n):
            env = rank_env(r, n, port, stencil_port)
            if env_fn is not None:
                env.update(env_fn(r))
            procs.append(subprocess.Popen(cmd, env=env, preexec_fn=_die_with_parent))
        t0 = time.monotonic()
        while True:
            codes = [p.poll() for p in procs]
            failed = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if failed:
                r, c = failed[0]
                rc = c if c > 0 else 128 - c
                print(f"[launch] rank {r} exited with {c}; stopping the other {n - 1} rank(s)", file=log, flush=True)
                _stop(procs)
                return rc
            if all(c == 0 for c in codes):
                return 0
            if timeout is not None and time.monotonic() - t0 > timeout:
                print(f"[launch] ranks still running after {timeout:.0f} s; stopping all {n}", file=log, flush=True)
                _stop(procs)
                return 124
            time.sleep(poll_s)
    except BaseException:  # KeyboardInterrupt / SIGTERM in the parent: take the ranks down too
        _stop(procs, grace=3.0)
        raise


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-n", "--nranks", type=int, required=True)
    ap.add_argument("--timeout", type=float, default=None, help="seconds before every rank is stopped (default: none)")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    cmd = a.cmd if not a.cmd[0].endswith(".py") else [sys.executable, *a.cmd]
    signal.signal(signal.SIGTERM, lambda *_: sys.exit(143))
    sys.exit(spawn_ranks(cmd, a.nranks, timeout=a.timeout))


if __name__ == "__main__":
    main()
