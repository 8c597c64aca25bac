"""Exchange-only timing split: blocking exchange()+swap() (bench_exchange definition) vs the same exchanges enqueued
stream-ordered with one sync at the end, on the 1-GPU 512^3 Jacobi3D domain (depth-2 halo, all self copies).
The difference is host round-trip cost per exchange; the stream-ordered number is the copy kernel's own rate."""
import json
import time

import torch

import stencil2_amd as st

L, N = 512, 50
m = st.Jacobi3D((L, L, L), gpus=[0], temporal=2)
m.init()
m.run(4)
m.synchronize()
dd = m.domain
dd.set_comm_max_blocks(0)
xb = dd.exchange_bytes_for_method(st.MethodFlags.All)
for _ in range(3):
    dd.exchange()
    dd.swap()
torch.cuda.synchronize()
out = {"bytes": xb}
for rep in range(2):
    t = time.perf_counter()
    for _ in range(N):
        dd.exchange()
        dd.swap()
    torch.cuda.synchronize()
    out[f"blocking_us_{rep}"] = (time.perf_counter() - t) / N * 1e6
    s = torch.cuda.Stream()  # not the null stream: exchange_async(0) means the domain's own comm streams
    t = time.perf_counter()
    for _ in range(N):
        dd.exchange_async(s.cuda_stream, 0)
        dd.swap()
    out[f"async_host_us_{rep}"] = (time.perf_counter() - t) / N * 1e6
    s.synchronize()
    out[f"async_us_{rep}"] = (time.perf_counter() - t) / N * 1e6
for k in list(out):
    if k.endswith(tuple("01")) and "host" not in k:
        out[k.replace("_us", "_GBps")] = round(xb / out[k] / 1e3, 1)
print(json.dumps(out), flush=True)
