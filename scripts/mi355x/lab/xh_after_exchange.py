"""Does the XH triple run slower right after the depth-3 exchange than back to back? 512^3 Jacobi with x read from
halos (bench.py's with-exchange model): 30 XH triples alone, then 30 x (exchange + XH triple), then 30 x (exchange
+ the whole-row triple). Run under rocprofv3 --kernel-trace and compare the kernel durations per phase (the field
is not swapped: the same input every launch).   python scripts/mi355x/lab/xh_after_exchange.py"""
import os
import sys

import torch

sys.path.append(os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
import stencil2_amd as st  # noqa: E402
from stencil2_amd import _C  # noqa: E402

m = st.Jacobi3D((512, 512, 512), gpus=[0], temporal=3, wrap_self=False, shared_halo_line=True, use_graph=False)
m.init()
m.run(6)
m.synchronize()
dd = m.domain
xh = _C.StencilTune()
xh.wrap = 0
wr = _C.StencilTune()
wr.wrap = 7
J = _C.StencilKind.Jacobi
for phase, exch, tune in (("xh_alone", False, xh), ("xh_after_exchange", True, xh), ("wrap_after_exchange", True, wr)):
    for _ in range(30):
        if exch:
            dd.exchange()
        assert _C.stencil7x3_apply(dd, 0, 0, J, True, 0, tune), phase
    torch.cuda.synchronize()
    print(phase, "done", flush=True)
