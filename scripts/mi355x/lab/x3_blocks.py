"""Per-block start / end of one fused-triple sweep (StencilTune.block_clock): which (z part, row group) blocks set the
sweep's time. python x3_blocks.py jacobi|astaroth NY [warm_triples] [x3sphw] [name=value ...] (StencilTune fields)

Blocks are printed per lockstep part (block lb = part * cm + row group); P is the one apply_x3_t's cost model picks
(stencil7x3.hip, x3sched 1), recomputed here for one MI355X (256 resident blocks) unless x3parts is given."""
import sys

import torch

import stencil2_amd as st

kind, ny = sys.argv[1], int(sys.argv[2])
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 4
sphw = float(sys.argv[4]) if len(sys.argv) > 4 else 0.3
clk = torch.zeros(1024, dtype=torch.int64, device="cuda")
t = st.StencilTune()
t.block_clock = clk.data_ptr()
t.x3sphw = sphw
Pshow, kw = 0, {}
for kv in sys.argv[5:]:
    k, v = kv.split("=", 1)
    if k == "P":  # the parts to print by (the host's plan may choose another P than the step-count model below)
        Pshow = int(v)
        continue
    if k == "xh":  # x read from exchanged halos (the XH kernel), as bench.py's with-exchange model
        kw = dict(wrap_self=not int(v), shared_halo_line=bool(int(v)))
        continue
    cur = getattr(t, k)
    setattr(t, k, (v.lower() in ("1", "true")) if isinstance(cur, bool) else type(cur)(v))
nz = 512
if kind == "jacobi":
    m = st.Jacobi3D((512, ny, nz), gpus=[0], temporal=3, tune=t, use_graph=False, **kw)
else:
    m = st.AstarothSim((512, ny, nz), gpus=[0], temporal=3, tune=t, quantities=1, use_graph=False, **kw)
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
cols, slots = (ny + 5) // 6, 256
P, best = Pshow or t.x3parts, 1e30
if P <= 0:
    for p in range(2, 9):
        cm = min(cols, slots // p)
        if cm < 1 or nz // p < 16:
            continue
        left = cols - cm
        cost = nz / p + 4 + (left * nz / (p * cm) + 4 if left > 0 else 0)
        if cost < best - 1e-9:
            best, P = cost, p
cm = nb // P
print(f"{kind} ny={ny} x3sphw={sphw} {' '.join(sys.argv[5:])}: {nb} blocks = {P} parts x {cm} groups "
      f"(+{cols - cm} leftover), sweep {max(en):.1f} us; block duration min {min(d):.1f} "
      f"median {sorted(d)[nb // 2]:.1f} max {max(d):.1f}; start skew max {max(st_):.1f}")
for q in range(P):
    row = [d[q * cm + col] for col in range(cm)]
    worst = sorted(range(cm), key=lambda col: -row[col])[:6]
    print(f"  part {q}: median {sorted(row)[cm // 2]:.1f} max {max(row):.1f} at groups {worst} ({', '.join('%.1f' % row[w] for w in worst)})")
    print("   ", " ".join("%.0f" % v for v in row))
