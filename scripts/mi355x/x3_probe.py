#!/usr/bin/env python3
"""Fused-triple probe: 512^3 (or --shape) Jacobi / Astaroth (one quantity) models with temporal=3, x wrapped in-kernel
(wrap 1) or every halo copied each triple (wrap 0: the XH triple reading x from 3-deep halos + the depth-3 exchange);
prints us per triple (hipGraph blocks, device-event timed) for each. Run under rocprofv3 --kernel-trace for the kernel
split.   python scripts/mi355x/x3_probe.py [--shape 512,512,512] [--kinds jacobi,astaroth] [--wraps 1,0] [--fp64]"""
import argparse
import json
import os
import sys
import time

import torch

# the repo's package unless PYTHONPATH names another copy (lab_alt/<name> for same-box A/B runs)
sys.path.append(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import stencil2_amd as st

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="512,512,512")
ap.add_argument("--kinds", default="jacobi,astaroth")
ap.add_argument("--wraps", default="1,0")
ap.add_argument("--fp64", action="store_true")
ap.add_argument("--steps", type=int, default=54)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--tune", default="", help="StencilTune fields name=value[,..]")
a = ap.parse_args()
shape = tuple(int(v) for v in a.shape.split(","))
for kind in a.kinds.split(","):
    for wrap in (int(v) for v in a.wraps.split(",")):
        t = st.StencilTune()
        for kv in filter(None, a.tune.split(",")):
            k, v = kv.split("=")
            cur = getattr(t, k)
            setattr(t, k, type(cur)(float(v)) if not isinstance(cur, bool) else bool(int(v)))
        kw = dict(gpus=[0], temporal=3, wrap_self=bool(wrap), tune=t, fp64=a.fp64, shared_halo_line=not wrap)
        m = st.Jacobi3D(shape, **kw) if kind == "jacobi" else st.AstarothSim(shape, quantities=1, **kw)
        m.init()
        m.prepare()
        m.run(a.steps)
        m.synchronize()
        best = 1e30
        for _ in range(a.rounds):
            t0 = time.perf_counter()
            m.run(a.steps)
            m.synchronize()
            best = min(best, (time.perf_counter() - t0) * 1e6 / a.steps)
        cells = shape[0] * shape[1] * shape[2]
        print(json.dumps({"kind": kind, "wrap": wrap, "fp64": a.fp64, "triples": m.temporal_triples(),
                          "wrap_axes": m.wrap_axes(), "us_per_step": round(best, 2),
                          "us_per_triple": round(3 * best, 1), "gcells": round(cells / best / 1e3, 1),
                          "halo_bytes": m.domain.exchange_bytes_for_method(st.MethodFlags.All)}), flush=True)
        del m
