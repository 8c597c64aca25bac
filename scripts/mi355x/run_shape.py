"""A few fused-pair steps of Jacobi3D on one sub-domain shape (one GPU, all halos periodic), for counter passes:
python3 scripts/mi355x/run_shape.py 645x645x323 --x2row 1 --steps 4"""
import argparse

import stencil2_amd as st

ap = argparse.ArgumentParser()
ap.add_argument("shape")
ap.add_argument("--x2row", type=int, default=1)
ap.add_argument("--steps", type=int, default=4)
ap.add_argument("--temporal", type=int, default=2)
args = ap.parse_args()
t = st.StencilTune()
t.x2row = args.x2row
m = st.Jacobi3D(tuple(int(v) for v in args.shape.split("x")), gpus=[0], temporal=args.temporal, tune=t,
                use_graph=False)
m.init()
m.run(args.steps)
m.synchronize()
print("ok", args.shape, "x2row", args.x2row, "wrap", m.wrap_axes())
