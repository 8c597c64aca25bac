#!/usr/bin/env python3
"""Parameterised GPU-box driver (replaces the round-1/2 single-use shell scripts).

Runs a list of steps on the gpurun box, each under its own time limit, with its output in <out>/<name>.log, and
stops at the first failing step (a GPU fault, abort or time limit ends the call: nothing else touches the GPU).
This process itself never initialises the GPU; every step is a child process.

    python3 scripts/mi355x/gpu.py --out gpurun_out/r3a  suite  bench  "mp:2:--steps 20 --colo-copy engine"
    python3 scripts/mi355x/gpu.py --out gpurun_out/r3b  "prof:b1:bench.py --steps 8"  "pmc:row:SQ_WAVES:bench.py --steps 4"

Steps:
    suite                 pytest -m gpu (whole suite, per-test thread timeout)
    tests:<expr>          pytest -m gpu -k <expr>
    ctest                 build/bin/stencil_ctest --gpu (native unit tests)
    bench[:<args>]        python bench.py <args> on the one GPU
    mp:<n>:<args>         torch.distributed.run with n ranks sharing the GPU: bench.py --gpus n <args>
    app:<name>:<args>     build/bin/<name> <args>
    prof:<name>:<cmd>     rocprofv3 --kernel-trace --stats around `python3 <cmd>` (one CSV set per process under
                          <out>/<name>)
    mpprof:<name>:<n>:<args>  same around an n-rank bench.py run
    pmc:<name>:<ctrs>:<cmd>   rocprofv3 --pmc <ctrs> (comma separated) around `python3 <cmd>`
    appprof:<name>:<app>:<args>  rocprofv3 --kernel-trace --stats around build/bin/<app> <args>
    apppmc:<name>:<ctrs>:<app>:<args>  rocprofv3 --pmc <ctrs> around build/bin/<app> <args>
    py:<script>:<args>    python3 <script> <args>
A step may start with environment assignments: "GPU_MAX_HW_QUEUES=2,STENCIL_LOG_LEVEL=3@mp:8:--per-gpu 128".
"""
from __future__ import annotations

import argparse
import glob
import os
import shlex
import shutil
import subprocess
import sys
import time

REPO = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
PY = sys.executable


def env():
    e = dict(os.environ)
    e.update({"STENCIL_SKIP_BUILD": "1", "STENCIL_PLAN_FILE": "0", "PYTHONPATH": REPO, "TMPDIR": "/tmp",
              "STENCIL_WAIT_TIMEOUT": e.get("STENCIL_WAIT_TIMEOUT", "30")})
    return e


def torchrun(n: int, port: int):
    return [PY, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}", "--master-addr=127.0.0.1",
            f"--master-port={port}"]


def step_cmd(step: str, out: str, k: int):
    kind, _, rest = step.partition(":")
    port = 29650 + 10 * k
    if kind == "suite":
        return "suite", [PY, "-u", "-m", "pytest", "tests", "-m", "gpu", "-x", "-q", "-p", "no:cacheprovider",
                         "--timeout", "200", "--timeout-method", "thread", "--durations=12"], 900
    if kind == "tests":
        return "tests", [PY, "-u", "-m", "pytest", "tests", "-m", "gpu", "-x", "-v", "-p", "no:cacheprovider",
                         "--timeout", "200", "--timeout-method", "thread", "-k", rest], 600
    if kind == "ctest":
        return "ctest", [os.path.join(REPO, "build/bin/stencil_ctest"), "--gpu"], 300
    if kind == "bench":
        return "bench", [PY, "bench.py", *shlex.split(rest)], 300
    if kind == "mp":
        n, _, args = rest.partition(":")
        return f"mp{n}", [*torchrun(int(n), port), "bench.py", "--gpus", n, *shlex.split(args)], 420
    if kind == "app":
        name, _, args = rest.partition(":")
        return f"app_{name}", [os.path.join(REPO, "build/bin", name), *shlex.split(args)], 300
    if kind == "py":
        script, _, args = rest.partition(":")
        return f"py_{os.path.basename(script).split('.')[0]}", [PY, script, *shlex.split(args)], 420
    if kind == "appprof":
        name, _, rest2 = rest.partition(":")
        app, _, args = rest2.partition(":")
        d = os.path.join(out, name)
        os.makedirs(d, exist_ok=True)
        pre = ["rocprofv3", "--kernel-trace", "--stats", "-d", d, "-o", "run_%pid%", "--output-format", "csv", "--"]
        return f"appprof_{name}", pre + [os.path.join(REPO, "build/bin", app), *shlex.split(args)], 300
    if kind == "apppmc":
        name, _, rest2 = rest.partition(":")
        ctrs, _, rest3 = rest2.partition(":")
        app, _, args = rest3.partition(":")
        d = os.path.join(out, name)
        os.makedirs(d, exist_ok=True)
        pre = ["rocprofv3", "--pmc", *ctrs.split(","), "--kernel-trace", "-d", d, "-o", "run_%pid%",
               "--output-format", "csv", "--"]
        return f"apppmc_{name}", pre + [os.path.join(REPO, "build/bin", app), *shlex.split(args)], 120
    if kind in ("prof", "mpprof", "pmc"):
        name, _, rest2 = rest.partition(":")
        d = os.path.join(out, name)
        os.makedirs(d, exist_ok=True)
        if kind == "pmc":
            ctrs, _, cmd = rest2.partition(":")
            pre = ["rocprofv3", "--pmc", *ctrs.split(","), "--kernel-trace", "-d", d, "-o", "run_%pid%",
                   "--output-format", "csv", "--"]
            return f"pmc_{name}", pre + [PY, *shlex.split(cmd)], 300
        pre = ["rocprofv3", "--kernel-trace", "--stats", "-d", d, "-o", "run_%pid%", "--output-format", "csv", "--"]
        if kind == "prof":
            return f"prof_{name}", pre + [PY, *shlex.split(rest2)], 420
        n, _, args = rest2.partition(":")
        return f"mpprof_{name}", pre + torchrun(int(n), port) + ["bench.py", "--gpus", n, *shlex.split(args)], 420
    raise SystemExit(f"unknown step {step!r}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("steps", nargs="+")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    os.chdir(REPO)
    for k, step in enumerate(a.steps):
        extra = {}
        if "@" in step.split(":")[0]:
            assigns, step = step.split("@", 1)
            extra = dict(kv.split("=", 1) for kv in assigns.split(","))
        name, cmd, limit = step_cmd(step, a.out, k)
        log = os.path.join(a.out, f"{k:02d}_{name}.log")
        print(f"[{time.strftime('%H:%M:%S')}] step {k}: {step} {extra or ''} (limit {limit} s) -> {log}", flush=True)
        t0 = time.time()
        with open(log, "w") as f:
            f.write(" ".join(shlex.quote(c) for c in cmd) + "\n")
            f.flush()
            try:
                rc = subprocess.run(["timeout", "-k", "10", str(limit), *cmd], stdout=f, stderr=subprocess.STDOUT,
                                    env={**env(), **extra}, cwd=REPO).returncode
            except Exception as e:  # noqa: BLE001
                rc = 99
                f.write(f"\nrunner error: {e}\n")
        dt = time.time() - t0
        with open(log) as f:
            lines = f.read().splitlines()
        keep = [ln for ln in lines if ln.startswith("{\"metric\"") or " passed" in ln or " failed" in ln
                or "error" in ln.lower()[:200]]
        for ln in (keep or lines[-5:])[-6:]:
            print("   ", ln[:1500], flush=True)
        for csv in sorted(glob.glob(os.path.join(a.out, "**", "*kernel_stats.csv"), recursive=True)):
            if os.path.getmtime(csv) >= t0:
                print("    stats:", csv, flush=True)
        print(f"    rc={rc} ({dt:.0f} s)", flush=True)
        if rc != 0:
            sys.exit(rc)
    shutil.rmtree(os.path.join(a.out, "__pycache__"), ignore_errors=True)


if __name__ == "__main__":
    main()
