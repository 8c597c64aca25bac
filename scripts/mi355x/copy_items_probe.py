"""Exchange-only time of the 512^3 radius-2-face self-exchange (bench_exchange config 3 on one GPU) for several copy
plan block sizes (items per 256-thread block for x-face rows / 16-B units), interleaved over rounds: blocking
exchange()+swap() and the same exchanges stream-ordered."""
import argparse
import json
import time

import torch

import stencil2_amd as st

ap = argparse.ArgumentParser()
ap.add_argument("--combos", default="1024:1024,256:1024,64:1024,1024:256,256:256")
ap.add_argument("--iters", type=int, default=40)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--edges", type=int, default=0, help="depth of the edge halos too (bench.py's fused pairs: 1)")
a = ap.parse_args()
r = st.Radius.constant(0)
r.set_face(2)
if a.edges:
    r.set_edge(a.edges)
combos = [tuple(int(v) for v in c.split(":")) for c in a.combos.split(",")]  # narrow:wide[:small_row_items]
doms = {}
for c in combos:
    n, w = c[0], c[1]
    st._C.set_copy_block_items(n, w)
    st._C.set_copy_small_rows(4096, c[2] if len(c) > 2 else 64)
    d = st.DistributedDomain(512, 512, 512, group=st.make_single_group())
    d.set_radius(r)
    d.set_gpus([0])
    d.add_data("q", torch.float32)
    d.realize()
    doms[c] = d
st._C.set_copy_block_items(1024, 512)  # the library defaults
st._C.set_copy_small_rows(4096, 64)
xs = torch.cuda.Stream()
best = {}
for rnd in range(a.rounds):
    for c, d in doms.items():
        for _ in range(3):
            d.exchange()
            d.swap()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            d.exchange()
            d.swap()
        blk = (time.perf_counter() - t) / a.iters * 1e6
        d.exchange_async(xs.cuda_stream, 0)
        xs.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            d.exchange_async(xs.cuda_stream, 0)
            d.swap()
        xs.synchronize()
        d.sync_exchange()
        asy = (time.perf_counter() - t) / a.iters * 1e6
        b = best.setdefault(c, [1e9, 1e9])
        b[0], b[1] = min(b[0], blk), min(b[1], asy)
xb = next(iter(doms.values())).exchange_bytes_for_method(st.MethodFlags.All)
for c, (blk, asy) in best.items():
    print(json.dumps({"narrow_items": c[0], "wide_items": c[1], "small_row_items": c[2] if len(c) > 2 else 64,  "block_us": round(blk, 1), "block_GBps": round(xb / blk / 1e3, 1),
                      "stream_us": round(asy, 1), "stream_GBps": round(xb / asy / 1e3, 1)}), flush=True)
