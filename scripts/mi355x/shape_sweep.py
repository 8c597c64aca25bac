"""Per-GPU throughput of the Jacobi3D step at the sub-domain shapes of the weak-scaling ladder, on ONE GPU (all
halos periodic self-copies): 512^3 (N=1), 645x323x645 (N=2), 813x407x407 (N=4), 1024x256x512 (N=8, 1x4x2) and
512^3 (N=8, 2x2x2). Separates the compute-shape cost from the communication cost of the multi-GPU runs."""
import argparse
import json
import time

import torch

import stencil2_amd as st

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=32)
ap.add_argument("--shapes", default="512x512x512,645x323x645,813x407x407,1024x256x512")
ap.add_argument("--x2sched", default="1")
ap.add_argument("--x2row", default="1,0", help="whole-row kernel on/off (StencilTune.x2row)")
ap.add_argument("--x2xfast", default="0", help="fused-pair column order: 1 x-major, 0 y-major (list)")
ap.add_argument("--interior-align", default="128", help="LocalDomain interior alignment in bytes (list: 64,128)")
ap.add_argument("--fp64", action="store_true")
ap.add_argument("--row-pad-lines", default="0", help="extra 128-B lines per row pitch (list)")
ap.add_argument("--altz", default="1", help="alternate the z-march direction every pair (list: 0,1)")
ap.add_argument("--temporal", type=int, default=2, help="steps fused per sweep (2 pairs, 3 triples)")
args = ap.parse_args()
for sched, row, xf, al, rp, az in ((int(a), int(b), int(c), int(e), int(f), int(h))
                                   for a in args.x2sched.split(",") for b in args.x2row.split(",")
                                   for c in args.x2xfast.split(",") for e in args.interior_align.split(",")
                                   for f in args.row_pad_lines.split(",") for h in args.altz.split(",")):
    for sh in args.shapes.split(","):
        L = tuple(int(v) for v in sh.split("x"))
        t = st.StencilTune()
        t.x2sched = sched
        t.x2row = row
        t.x2xfast = xf
        t.alternate_z = bool(az)
        m = st.Jacobi3D(L, gpus=[0], temporal=args.temporal, tune=t, interior_align=al, fp64=args.fp64, row_pad_lines=rp)
        m.init()
        m.prepare()  # graph blocks instantiated outside the timed region (the first instantiation in a process is slow)
        m.run(8)
        m.synchronize()
        t0 = time.perf_counter()
        m.run(args.steps)
        m.synchronize()
        dt = time.perf_counter() - t0
        cells = L[0] * L[1] * L[2]
        print(json.dumps({"shape": sh, "x2sched": sched, "x2row": row, "x2xfast": xf, "interior_align": al, "row_pad_lines": rp, "altz": az,
                          "temporal": 3 if m.temporal_triples() else 2, "wrap_axes": m.wrap_axes(), "fp64": args.fp64, "us_per_step": round(dt / args.steps * 1e6, 1),
                          "gcells": round(cells * args.steps / dt / 1e9, 1)}), flush=True)
        del m
        torch.cuda.empty_cache()
