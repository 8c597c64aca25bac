"""Per-block start / end of one fused-triple sweep (StencilTune.block_clock): which (z part, row group) blocks set the
sweep's time. python x3_blocks.py jacobi|astaroth NY [warm_triples]"""
import sys

import torch

import stencil2_amd as st

kind, ny = sys.argv[1], int(sys.argv[2])
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 4
sphw = float(sys.argv[4]) if len(sys.argv) > 4 else 0.75
clk = torch.zeros(1024, dtype=torch.int64, device="cuda")
t = st.StencilTune()
t.block_clock = clk.data_ptr()
t.x3sphw = sphw
if kind == "jacobi":
    m = st.Jacobi3D((512, ny, 512), gpus=[0], temporal=3, tune=t, use_graph=False)
else:
    m = st.AstarothSim((512, ny, 512), gpus=[0], temporal=3, tune=t, quantities=1, use_graph=False)
m.init()
assert m.temporal_triples()
for i in range(warm + 1):
    clk.zero_()
    m.run(3)
    m.synchronize()
c = clk.view(-1, 2).cpu()
used = (c[:, 1] > 0).nonzero().flatten()
nb = int(used.max()) + 1
t0 = int(c[used, 0].min())
d = [(int(c[b, 1]) - int(c[b, 0])) / 100.0 for b in range(nb)]  # 100 MHz wall clock -> us
st_ = [(int(c[b, 0]) - t0) / 100.0 for b in range(nb)]
en = [(int(c[b, 1]) - t0) / 100.0 for b in range(nb)]
P = 3
cm = nb // P
print(f"{kind} ny={ny} x3sphw={sphw}: {nb} blocks, sweep {max(en):.1f} us; block duration min {min(d):.1f} median {sorted(d)[nb // 2]:.1f} max {max(d):.1f}; start skew max {max(st_):.1f}")
for q in range(P):
    row = [d[q * cm + col] for col in range(cm)]
    worst = sorted(range(cm), key=lambda col: -row[col])[:6]
    print(f"  part {q}: median {sorted(row)[cm // 2]:.1f} max {max(row):.1f} at groups {worst} ({', '.join('%.1f' % row[w] for w in worst)})")
    print("   ", " ".join("%.0f" % v for v in row))
