"""Blocking exchange()+swap() latency on one GPU, split by host-side mechanism (bench_exchange definition).

For a 512^3 fp32 domain (radius given by --radius: 'faces2' = bench_exchange config 3, 'bench' = bench.py's depth-2
faces + depth-1 edges) time, interleaved over rounds:
  block      hipDeviceSynchronize before, hipStreamSynchronize after   (spin_wait off, null_stream_producers off)
  spin       host spins on a host-mapped epoch word, then synchronizes (spin_wait on)
  null       comm stream waits on a null-stream event instead of hipDeviceSynchronize (null_stream_producers on)
  spin+null  both
  async      the same exchanges stream-ordered back to back (exchange_async on a caller stream), one sync at the end
"""
import argparse
import json
import time

import torch

import stencil2_amd as st

ap = argparse.ArgumentParser()
ap.add_argument("--size", type=int, default=512)
ap.add_argument("--radius", default="faces2")
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--schedule", default="", help="hipSetDeviceFlags host wait policy before the GPU is used: spin/yield/blocking/auto")
ap.add_argument("--only", default="", help="comma list of modes (block,spin,null,spin+null); sector A/B off")
a = ap.parse_args()
if a.schedule:
    err = st._C.set_device_schedule(a.schedule)
    print("schedule", a.schedule, err or "ok")

r = st.Radius.constant(0)
r.set_face(2)
if a.radius == "bench":
    r.set_edge(1)


def make(sectors):
    d = st.DistributedDomain(a.size, a.size, a.size, group=st.make_single_group())
    d.set_radius(r)
    d.set_gpus([0])
    tr = st.TransportOptions()
    tr.x_face_sectors = sectors
    d.set_transport_options(tr)
    d.add_data("d", torch.float32)
    d.realize()
    return d


doms = {"": make(False)} if a.only else {"": make(False), "sect/": make(True)}
xb = doms[""].exchange_bytes_for_method(st.MethodFlags.All)


def setmode(dd, spin, null):
    o = dd.transport_options()
    o.spin_wait = spin
    o.null_stream_producers = null
    dd.set_transport_options_live(o)


res = {}
for rnd in range(a.rounds):
  for pre, dd in doms.items():
    for name, spin, null in (("block", False, False), ("spin", True, False), ("null", False, True),
                             ("spin+null", True, True)):
        if a.only and name not in a.only.split(","):
            continue
        name = pre + name
        setmode(dd, spin, null)
        for _ in range(5):
            dd.exchange()
            dd.swap()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            dd.exchange()
            dd.swap()
        dt = (time.perf_counter() - t) / a.iters
        res.setdefault(name, []).append(dt)
    s = torch.cuda.Stream()
    for _ in range(5):
        dd.exchange_async(s.cuda_stream, 0)
        dd.swap()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.iters):
        dd.exchange_async(s.cuda_stream, 0)
        dd.swap()
    s.synchronize()
    dd.sync_exchange()
    res.setdefault(pre + "async", []).append((time.perf_counter() - t) / a.iters)

out = {"size": a.size, "radius": a.radius, "bytes": xb, "schedule": a.schedule or "default"}
for k, v in res.items():
    out[k] = {"us": round(min(v) * 1e6, 2), "us_all": [round(x * 1e6, 2) for x in v], "GBps": round(xb / min(v) / 1e9, 1)}
print(json.dumps(out))
