"""Jacobi3D / Astaroth proxy on the CPU backend vs the pure-torch oracle (bitwise, same operation order)."""
import os

import pytest
import torch

from stencil2_amd.ops import astaroth_init_reference, astaroth_step_reference, jacobi_step_reference


def gather(model):
    dd = model.domain
    L = dd.size()
    g = None
    for di in range(dd.num_domains()):
        d = dd.domain(di)
        o, s = d.origin(), d.size()
        t = model.interior(di)
        if g is None:
            g = torch.zeros(L.z, L.y, L.x, dtype=t.dtype)
        g[o.z:o.z + s.z, o.y:o.y + s.y, o.x:o.x + s.x] = t
    return g


@pytest.mark.parametrize("gpus", [[0], [0, 0, 0]])
@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("fp64", [False, True])
def test_jacobi_host_matches_oracle(st, gpus, overlap, fp64):
    m = st.Jacobi3D((21, 17, 15), gpus=gpus, backend=st.Backend.Host, overlap=overlap, fp64=fp64)
    m.init()
    u = gather(m)
    assert float(u.mean()) == 0.5
    for _ in range(4):
        m.step()
        u = jacobi_step_reference(u)
    m.synchronize()
    assert torch.equal(gather(m), u)


def test_astaroth_host_matches_oracle(st):
    L = (18, 16, 14)
    m = st.AstarothSim(L, quantities=2, gpus=[0], backend=st.Backend.Host)
    m.init()
    u0 = astaroth_init_reference(L, 3, 10.0)
    assert torch.allclose(gather(m), u0, atol=1e-6)
    u = gather(m)
    for _ in range(3):
        m.step()
        u = astaroth_step_reference(u)
    m.synchronize()
    assert torch.equal(gather(m), u)


def test_paraview_roundtrip(st, tmp_path):
    from stencil2_amd.utils import read_paraview

    m = st.Jacobi3D((6, 5, 4), gpus=[0, 0], backend=st.Backend.Host)
    m.init()
    m.step()
    m.synchronize()
    prefix = str(tmp_path / "jac")
    m.domain.write_paraview(prefix)
    cols = read_paraview(prefix)
    assert list(cols.keys())[:4] == ["Z", "Y", "X", "d"]  # names preserved (reference bug §2.6-6)
    assert len(cols["X"]) == 6 * 5 * 4
    g = gather(m)
    for z, y, x, v in zip(cols["Z"], cols["Y"], cols["X"], cols["d"]):
        assert abs(float(g[z, y, x]) - v) < 1e-6


def test_checkpoint_resume_bitwise(st, tmp_path):
    """save -> keep stepping -> restore -> re-step: identical trajectory (binary per-sub-domain checkpoints)."""
    m = st.Jacobi3D((20, 14, 12), gpus=[0, 0], backend=st.Backend.Host)
    m.init()
    m.run(2)
    m.synchronize()
    prefix = str(tmp_path / "ck")
    m.domain.save_checkpoint(prefix)
    m.run(3)
    m.synchronize()
    ref = gather(m).clone()
    m2 = st.Jacobi3D((20, 14, 12), gpus=[0, 0], backend=st.Backend.Host)
    m2.init()
    m2.domain.load_checkpoint(prefix)
    m2.run(3)
    m2.synchronize()
    assert torch.equal(gather(m2), ref)
    m3 = st.Jacobi3D((20, 14, 10), gpus=[0, 0], backend=st.Backend.Host)
    m3.init()
    with pytest.raises(RuntimeError):
        m3.domain.load_checkpoint(prefix)
