"""Launch N ranks of a native app or Python script on this node (an `mpirun -n` equivalent for the TCP
process group): python -m stencil2_amd.launch -n 4 build/bin/jacobi3d 256 256 256 -n 20"""
from __future__ import annotations

import argparse
import os
import socket
import subprocess
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-n", "--nranks", type=int, required=True)
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(a.nranks):
        env = dict(os.environ, STENCIL_RANK=str(r), STENCIL_WORLD_SIZE=str(a.nranks), STENCIL_MASTER_ADDR="127.0.0.1",
                   STENCIL_MASTER_PORT=str(port), LOCAL_RANK=str(r))
        cmd = a.cmd if not a.cmd[0].endswith(".py") else [sys.executable, *a.cmd]
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    for p in procs:
        rc = max(rc, p.wait())
    sys.exit(rc)


if __name__ == "__main__":
    main()
