"""Fused-triple kernel time vs grid rows / halo radius: python x3_radius.py NX NY NZ RADIUS [steps] [kind]"""
import sys

import stencil2_amd as st

nx, ny, nz, rad = (int(v) for v in sys.argv[1:5])
steps = int(sys.argv[5]) if len(sys.argv) > 5 else 36
kind = sys.argv[6] if len(sys.argv) > 6 else "jacobi"
if kind == "jacobi":
    m = st.StencilModel((nx, ny, nz), kind=st.StencilKind.Jacobi, radius=rad, temporal=3, gpus=[0])
else:
    m = st.AstarothSim((nx, ny, nz), quantities=1, temporal=3, gpus=[0])
m.init()
assert m.temporal_triples()
m.prepare()
m.run(steps)
m.synchronize()
d = m.domain.domain(0)
print("ok", nx, ny, nz, rad, kind, "pitch", d.pitch(0), "raw", d.raw_size())
