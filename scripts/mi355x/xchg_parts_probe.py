"""Stream-ordered self-exchange time per halo part (x faces, y faces, z faces, edges, corners, all 26 directions) of
one periodic sub-domain on one GPU: which part of a BASELINE exchange config (default: config 5a's 1024^3 fp64,
radius 3, one quantity) the copy-plan kernel spends its time on. Prints one JSON line per part."""
import argparse
import json
import time

import torch

import stencil2_amd as st

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1024)
ap.add_argument("--x-face-sectors", type=int, default=0, help="TransportOptions.x_face_sectors")
ap.add_argument("--shape", default="", help="x,y,z instead of the --n cube")
ap.add_argument("--radius", type=int, default=3)
ap.add_argument("--fp64", type=int, default=1)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--parts", default="x,y,z,faces,all")
ap.add_argument("--narrow", default="1024", help="comma list: x-face rows per block (set_copy_block_items)")
a = ap.parse_args()
R = a.radius
X, Y, Z = (int(v) for v in a.shape.split(",")) if a.shape else (a.n, a.n, a.n)


def radius_for(part):
    r = st.Radius.constant(0)
    for dx in (-1, 0, 1):
        for dy in (-1, 0, 1):
            for dz in (-1, 0, 1):
                k = abs(dx) + abs(dy) + abs(dz)
                if k == 0:
                    continue
                on = {"x": k == 1 and dx != 0, "y": k == 1 and dy != 0, "z": k == 1 and dz != 0, "faces": k == 1,
                      "edges": k == 2, "corners": k == 3, "all": True}[part]
                if on:
                    r.set_dir(dx, dy, dz, R)
    return r


dt = torch.float64 if a.fp64 else torch.float32
xs = torch.cuda.Stream()
for part, narrow in [(p, int(n)) for n in a.narrow.split(",") for p in a.parts.split(",")]:
    st._C.set_copy_block_items(narrow, 512)
    d = st.DistributedDomain(X, Y, Z, group=st.make_single_group())
    d.set_radius(radius_for(part))
    topt = st.TransportOptions()
    topt.x_face_sectors = bool(a.x_face_sectors)
    d.set_transport_options(topt)
    d.set_gpus([0])
    d.add_data("q", dt)
    d.realize()
    for _ in range(3):
        d.exchange()
        d.swap()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.iters):
        d.exchange_async(xs.cuda_stream, 0)
        d.swap()
    xs.synchronize()
    d.sync_exchange()
    us = (time.perf_counter() - t) / a.iters * 1e6
    b = d.exchange_bytes_for_method(st.MethodFlags.All)
    print(json.dumps({"part": part, "narrow": narrow, "shape": [X, Y, Z], "radius": R, "fp64": bool(a.fp64), "x_face_sectors": a.x_face_sectors, "bytes": b, "us": round(us, 1),
                      "GBps": round(b / us / 1e3, 1)}), flush=True)
    del d
    torch.cuda.empty_cache()
