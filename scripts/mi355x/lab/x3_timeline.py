"""Fused-triple dispatch times over a long run (data / clock drift): python x3_timeline.py jacobi|astaroth STEPS"""
import sys

import stencil2_amd as st

kind, steps = sys.argv[1], int(sys.argv[2])
m = (st.Jacobi3D((512, 512, 512), gpus=[0], temporal=3) if kind == "jacobi"
     else st.AstarothSim((512, 512, 512), gpus=[0], temporal=3, quantities=1))
m.init()
assert m.temporal_triples()
m.prepare()
m.run(steps)
m.synchronize()
print("ok", kind, steps)
