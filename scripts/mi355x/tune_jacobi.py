"""Correctness + sweep of StencilTune knobs for the 1-GPU Jacobi3D step (interleaved rounds in one process)."""
import json
import sys
import time

import torch

import stencil2_amd as st
from stencil2_amd.ops import jacobi_step_reference


def tune(variant, ty, zc, nt=True, remap=True):
    t = st.StencilTune()
    t.variant, t.ty, t.zchunk, t.nontemporal, t.xcd_remap = variant, ty, zc, nt, remap
    return t


def check(t, size, overlap):
    m = st.Jacobi3D(size, gpus=[0], tune=t, overlap=overlap, auto_overlap=False)
    m.init()
    u = m.interior().clone().cpu()
    for _ in range(3):
        m.step()
        u = jacobi_step_reference(u)
    m.synchronize()
    got = m.interior().cpu()
    return torch.equal(got, u)


def timeit(t, L, steps, overlap=True):
    m = st.Jacobi3D((L, L, L), gpus=[0], tune=t, overlap=overlap, auto_overlap=False)
    m.init()
    m.run(3)
    m.synchronize()
    t0 = time.perf_counter()
    m.run(steps)
    m.synchronize()
    dt = (time.perf_counter() - t0) / steps
    del m
    torch.cuda.empty_cache()
    return dt


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    variants = [(0, 4, 0), (0, 4, 24), (0, 2, 0), (0, 8, 0), (1, 4, 16)]
    ok = True
    for v in variants:
        for size in [(67, 45, 33), (64, 64, 64)]:
            for ov in (True, False):
                good = check(tune(*v), size, ov)
                ok &= good
                if not good:
                    print(json.dumps({"variant": v, "size": size, "overlap": ov, "correct": False}), flush=True)
    print(json.dumps({"all_correct": ok}), flush=True)
    res = {(v, ov): [] for v in variants for ov in (True, False)}
    for rnd in range(2):
        for v in variants:
            for ov in (True, False):
                res[(v, ov)].append(timeit(tune(*v), L, 20, ov))
    for (v, ov), ts in res.items():
        best = min(ts)
        print(json.dumps({"variant": v[0], "ty": v[1], "zchunk": v[2], "overlap": ov, "ms": round(best * 1e3, 4),
                          "gcells": round(L ** 3 / best / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
