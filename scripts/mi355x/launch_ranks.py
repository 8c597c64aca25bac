#!/usr/bin/env python3
"""Start N ranks of a command on this node with the torch.distributed / native-group rendezvous environment,
substituting {rank} in the command's arguments (e.g. per-rank rocprofv3 output directories):

    python scripts/mi355x/launch_ranks.py -n 2 --timeout 300 -- rocprofv3 --kernel-trace --stats \
        -d gpurun_out/prof/rank{rank} -- python3 bench.py --gpus 2 --steps 10

Stdlib only and GPU-free: it loads stencil2_amd/launch.py by path (not the package, whose import loads torch and the
HIP runtime), so every rank is a fresh child of a process that never touched the GPU -- under rocprofv3 each rank is
its own profiled program, and no profiled process forks another."""
import argparse
import importlib.util
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-n", type=int, required=True)
    ap.add_argument("--timeout", type=float, default=None)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    spec = importlib.util.spec_from_file_location("_l", os.path.join(REPO, "stencil2_amd", "launch.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    port = m.free_port()
    procs_rc = []
    # spawn_ranks runs one command for all ranks; {rank} differs per rank, so start them through a per-rank env hook
    # and a tiny shim that formats the command with the rank it was given
    shim = [sys.executable, "-c",
            "import os,sys,subprocess; r=os.environ['RANK']; "
            "sys.exit(subprocess.call([x.replace('{rank}', r) for x in sys.argv[1:]]))", *cmd]
    sys.exit(m.spawn_ranks(shim, a.n, timeout=a.timeout, port=port))


if __name__ == "__main__":
    main()
