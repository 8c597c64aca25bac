"""Diagnose the overlapped fused pair: which cells differ from the oracle after one pair."""
import sys
import torch
import stencil2_amd as st
from stencil2_amd.ops import jacobi_step_reference

sys.path.insert(0, "tests")
from test_gpu import _gather  # noqa: E402

for methods in ["Kernel"]:
    for gpus in ([0],):
        m = st.Jacobi3D((40, 36, 44), gpus=gpus, methods=getattr(st.MethodFlags, methods), temporal=2, overlap=True,
                        auto_overlap=False)
        m.init()
        u = _gather(m)
        m.run(2)
        m.synchronize()
        g = _gather(m)
        u1 = jacobi_step_reference(u)
        want = jacobi_step_reference(u1)
        bad = (g != want)
        idx = bad.nonzero()
        print(methods, gpus, "bad", int(bad.sum()), flush=True)
        for (z, y, x) in idx[:: max(1, len(idx) // 12)].tolist()[:12]:
            print((z, y, x), "got", float(g[z, y, x]), "want", float(want[z, y, x]), "u1", float(u1[z, y, x]),
                  "u0", float(u[z, y, x]))
        # which slabs
        inner = torch.zeros_like(bad)
        inner[2:-2, 2:-2, 2:-2] = True
        print("bad inside interior", int((bad & inner).sum()), "bad in exterior", int((bad & ~inner).sum()),
              "exterior cells", int((~inner).sum()))
        print("full field curr after:", m.field(0).shape, float(m.field(0).float().abs().max()))
