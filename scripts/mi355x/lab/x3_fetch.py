"""One fused-triple model for kernel-trace / PMC runs:
    python x3_fetch.py NX NY NZ [x3sched] [x3parts] [steps] [row_pad_lines] [shared_halo_line]"""
import sys

import stencil2_amd as st

nx, ny, nz = (int(v) for v in sys.argv[1:4])
sched = int(sys.argv[4]) if len(sys.argv) > 4 else 1
parts = int(sys.argv[5]) if len(sys.argv) > 5 else 0
steps = int(sys.argv[6]) if len(sys.argv) > 6 else 36
pad = int(sys.argv[7]) if len(sys.argv) > 7 else 0
shared = bool(int(sys.argv[8])) if len(sys.argv) > 8 else False
t = st.StencilTune()
t.x3sched = sched
t.x3parts = parts
m = st.Jacobi3D((nx, ny, nz), gpus=[0], temporal=3, tune=t, row_pad_lines=pad, shared_halo_line=shared)
m.init()
assert m.temporal_triples()
m.prepare()
m.run(steps)
m.synchronize()
d = m.domain.domain(0)
print("ok", nx, ny, nz, sched, parts, steps, "pitch", d.pitch(0), "raw", d.raw_size())
