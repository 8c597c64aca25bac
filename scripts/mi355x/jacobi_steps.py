"""Minimal driver for counter collection: init + N Jacobi steps on one GPU (+ a torch copy roofline)."""
import sys
import time
import torch
import stencil2_amd as st

L = int(sys.argv[1]) if len(sys.argv) > 1 else 512
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
overlap = (sys.argv[3] != "0") if len(sys.argv) > 3 else True
t = st.StencilTune()
if len(sys.argv) > 4:
    t.variant, t.ty, t.zchunk = (int(v) for v in sys.argv[4].split(","))
m = st.Jacobi3D((L, L, L), gpus=[0], overlap=overlap, auto_overlap=False, tune=t)
m.init()
m.run(n)
m.synchronize()
del m
# roofline reference: device copy of the same byte count
a = torch.empty(L * L * L, dtype=torch.float32, device="cuda")
b = torch.empty_like(a)
for _ in range(3):
    b.copy_(a)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(10):
    b.copy_(a)
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / 10
print("torch copy", L ** 3 * 8 / dt / 1e12, "TB/s", dt * 1e6, "us")
