"""GPU (MI355X) tests: every transport on the device backend against the coordinate oracle, the HIP stencil kernels
against the torch fp32/fp64 oracle (bitwise), multi-process HIP-IPC on one GPU (reference
test_cuda_mpi_colocatedtx.cu runs both ranks on device 0 the same way)."""
import os

import pytest
import torch

from conftest import run_ranks
from stencil2_amd.ops import astaroth_init_reference, astaroth_step_reference, jacobi_step_reference
from stencil2_amd.utils.testing import check_exchange, fill_coords

pytestmark = pytest.mark.gpu
WORKER = os.path.join(os.path.dirname(__file__), "mp_worker.py")


def _dd(st, size, radius, gpus, methods, dtype=torch.int64, transport=None):
    dd = st.DistributedDomain(*size, group=st.make_single_group())
    dd.set_backend(st.Backend.Device)
    if transport is not None:
        dd.set_transport_options(transport)
    dd.set_radius(radius)
    dd.set_gpus(gpus)
    dd.set_methods(methods)
    q = dd.add_data("c", dtype)
    dd.realize()
    return dd, q


def _radii(st):
    a = st.Radius.constant(0)
    a.set_dir(1, 0, 0, 2)
    a.set_dir(-1, 0, 0, 1)
    b = st.Radius.constant(1)
    b.set_dir(0, 0, 1, 3)
    return {"r1": st.Radius.constant(1), "r3": st.Radius.constant(3), "asym": a, "fec": st.Radius.face_edge_corner(2, 1, 1),
            "mixed": b}


@pytest.mark.parametrize("method,gpus", [("Kernel", [0]), ("Kernel", [0, 0]), ("PeerCopy", [0, 0]),
                                         ("PeerCopyEngine", [0, 0]), ("PeerCopyEngine", [0, 0, 0]),
                                         ("PeerCopyPeerApi", [0, 0]), ("PeerCopyPeerApi", [0, 0, 0]),
                                         ("Rccl", [0, 0]), ("Staged", [0, 0]), ("All", [0, 0, 0])])
@pytest.mark.parametrize("rname", ["r1", "r3", "asym", "fec", "mixed"])
def test_device_exchange(st, method, gpus, rname):
    """PeerCopyEngine: PeerCopy messages between sub-domains packed, copied by a DMA engine, unpacked
    (TransportOptions.peer_copy = Engine; self-neighbour messages stay direct stores). PeerCopyPeerApi: the same
    pipes through hipMemcpyPeerAsync(dst, dev, src, dev) -- the cross-GPU call of the reference's PeerCopySender
    (tx_cuda.cuh:153), executed with both ends on device 0."""
    radius = _radii(st)[rname]
    tr = st.TransportOptions()
    if method in ("PeerCopyEngine", "PeerCopyPeerApi"):
        tr.peer_copy = st.TransportOptions.Copy.Engine
        tr.peer_api_same_device = method == "PeerCopyPeerApi"
        method = "PeerCopy"
    dd, q = _dd(st, (19, 13, 11), radius, gpus, getattr(st.MethodFlags, method), transport=tr)
    for it in range(2):
        fill_coords(dd, q)
        dd.exchange()
        assert check_exchange(dd, q, radius) == 0
        dd.swap()


@pytest.mark.parametrize("method,gpus", [("Kernel", [0]), ("Kernel", [0, 0]), ("PeerCopy", [0, 0]),
                                         ("PeerCopyEngine", [0, 0]), ("Rccl", [0, 0]), ("Staged", [0, 0])])
@pytest.mark.parametrize("rname", ["r1", "r3", "asym", "fec"])
def test_device_exchange_shared_halo_lines(st, method, gpus, rname):
    """Shared halo lines (row r's +x and row r+1's -x halo in one 128-B line) on the device backend: every transport
    against the coordinate oracle, fp32 and int64 rows long enough for whole lines."""
    radius = _radii(st)[rname]
    tr = st.TransportOptions()
    if method == "PeerCopyEngine":
        tr.peer_copy = st.TransportOptions.Copy.Engine
        method = "PeerCopy"
    for dtype in (torch.float32, torch.int64):
        dd = st.DistributedDomain(96, 13, 11, group=st.make_single_group())
        dd.set_backend(st.Backend.Device)
        dd.set_transport_options(tr)
        dd.set_radius(radius)
        dd.set_gpus(gpus)
        dd.set_methods(getattr(st.MethodFlags, method))
        dd.set_shared_halo_line(True)
        q = dd.add_data("c", dtype)
        dd.realize()
        assert all(dd.domain(i).shared_halo_line() for i in range(dd.num_domains()))
        for it in range(2):
            fill_coords(dd, q, offset=it)
            dd.exchange()
            assert check_exchange(dd, q, radius, offset=it) == 0
            dd.swap()


@pytest.mark.parametrize("kind,size,temporal", [("jacobi", (512, 120, 116), 2), ("jacobi", (512, 120, 116), 1),
                                                ("astaroth", (512, 36, 28), 2), ("astaroth", (256, 24, 20), 1)])
def test_shared_halo_lines_models_match_oracle(st, kind, size, temporal):
    """Fused pairs / single steps on the shared-halo-line layout with every halo copied (wrap_self=False, config 2
    as defined) and with in-kernel wrap: bitwise equal to the torch oracle."""
    from stencil2_amd.ops import astaroth_step_reference
    cls, ref, kw = ((st.Jacobi3D, jacobi_step_reference, {}) if kind == "jacobi"
                    else (st.AstarothSim, astaroth_step_reference, {"quantities": 2}))
    for wrap in (False, True):
        m = cls(size, gpus=[0], temporal=temporal, wrap_self=wrap, shared_halo_line=True, **kw)
        m.init()
        assert m.domain.domain(0).shared_halo_line()
        u = torch.rand((size[2], size[1], size[0]), device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
        for q in range(kw.get("quantities", 1)):
            m.interior(0, q).copy_(u)
        torch.cuda.synchronize()
        m.run(5)
        for _ in range(5):
            u = ref(u)
        m.synchronize()
        for q in range(kw.get("quantities", 1)):
            assert torch.equal(m.interior(0, q), u), f"wrap_self={wrap} q{q}"


@pytest.mark.parametrize("reserve", [8, 0, 32])
def test_astaroth_forced_overlap_one_gpu(st, reserve):
    """Config 4 as the reference iterates (bin/astaroth_sim.cu:223-274) on one GPU: interior sweep overlapped with
    the same-GPU radius-3 exchange (the translate confined to `reserve` CUs the sweep leaves free; 0 = unconfined),
    exterior slabs after; every halo copied (wrap_self=False). Bitwise equal to the oracle."""
    from stencil2_amd.ops import astaroth_step_reference
    t = st.StencilTune()
    t.x2reserve = reserve
    size = (64, 40, 36)
    m = st.AstarothSim(size, quantities=2, gpus=[0], overlap=True, auto_overlap=False, wrap_self=False, tune=t)
    m.init()
    assert m.overlapping()
    u = torch.rand((size[2], size[1], size[0]), device="cuda", generator=torch.Generator(device="cuda").manual_seed(9))
    for q in range(2):
        m.interior(0, q).copy_(u)
    torch.cuda.synchronize()
    m.run(4)
    for _ in range(4):
        u = astaroth_step_reference(u)
    m.synchronize()
    for q in range(2):
        assert torch.equal(m.interior(0, q), u)


def test_device_exchange_float_views(st):
    radius = st.Radius.constant(2)
    dd, q = _dd(st, (64, 32, 16), radius, [0], st.MethodFlags.All, dtype=torch.float32)
    t = dd.curr(0, q)
    assert t.device.type == "cuda" and t.dtype == torch.float32
    fill_coords(dd, q)
    dd.exchange()
    assert check_exchange(dd, q, radius) == 0


def _gather(model, q=0):
    dd = model.domain
    L = dd.size()
    g = None
    for di in range(dd.num_domains()):
        d = dd.domain(di)
        o, s = d.origin(), d.size()
        t = model.interior(di, q).cpu()
        if g is None:
            g = torch.zeros(L.z, L.y, L.x, dtype=t.dtype)
        g[o.z:o.z + s.z, o.y:o.y + s.y, o.x:o.x + s.x] = t
    return g


@pytest.mark.parametrize("size", [(32, 32, 32), (67, 45, 33), (130, 64, 40)])
@pytest.mark.parametrize("gpus", [[0], [0, 0]])
@pytest.mark.parametrize("overlap", [True, False])
@pytest.mark.parametrize("variant", [0, 1, 2, 3])
def test_jacobi_device_matches_oracle(st, size, gpus, overlap, variant):
    """exchange + stencil pipelines (forwarding off): overlap (interior/exchange/exterior) and whole-region."""
    t = st.StencilTune()
    t.variant = variant
    m = st.Jacobi3D(size, gpus=gpus, overlap=overlap, auto_overlap=False, tune=t, forward=False)
    m.init()
    assert not m.forwarding()
    u = _gather(m)
    for _ in range(3):
        m.step()
        u = jacobi_step_reference(u)
    m.synchronize()
    assert torch.equal(_gather(m), u)


def _check_halos(model, g, radius_dirs):
    """Every halo cell in a direction with a message holds its periodic image of the global field g."""
    from stencil2_amd.ops import periodic_gather
    dd = model.domain
    bad = 0
    for di in range(dd.num_domains()):
        d = dd.domain(di)
        o, raw = d.accessor_origin(), d.raw_size()
        full = model.field(di).cpu()
        want = periodic_gather(g, (o.x, o.y, o.z), (raw.x, raw.y, raw.z))
        cr = d.get_compute_region()
        gz = torch.arange(raw.z).view(-1, 1, 1) + o.z
        gy = torch.arange(raw.y).view(1, -1, 1) + o.y
        gx = torch.arange(raw.x).view(1, 1, -1) + o.x
        dz = (gz >= cr.hi.z).long() - (gz < cr.lo.z).long()
        dy = (gy >= cr.hi.y).long() - (gy < cr.lo.y).long()
        dx = (gx >= cr.hi.x).long() - (gx < cr.lo.x).long()
        dz, dy, dx = torch.broadcast_tensors(dz, dy, dx)
        mask = torch.zeros(full.shape, dtype=torch.bool)
        for (xx, yy, zz) in radius_dirs:
            mask |= (dx == xx) & (dy == yy) & (dz == zz)
        bad += int((full[mask] != want[mask]).sum())
    return bad


_FACES = [(1, 0, 0), (-1, 0, 0), (0, 1, 0), (0, -1, 0), (0, 0, 1), (0, 0, -1)]
_ALL26 = [(x, y, z) for z in (-1, 0, 1) for y in (-1, 0, 1) for x in (-1, 0, 1) if (x, y, z) != (0, 0, 0)]


@pytest.mark.parametrize("size", [(32, 32, 32), (67, 45, 33), (130, 64, 40)])
@pytest.mark.parametrize("gpus,methods", [([0], "All"), ([0, 0], "All"), ([0, 0, 0, 0], "All"), ([0, 0], "PeerCopy")])
@pytest.mark.parametrize("fp64", [False, True])
def test_jacobi_forwarding_matches_oracle(st, size, gpus, methods, fp64):
    """Halo forwarding: the stencil kernel writes the receivers' halos (Kernel/PeerCopy targets); results stay
    bitwise equal to the oracle and the new curr halos are valid after every step without any exchange()."""
    m = st.Jacobi3D(size, gpus=gpus, fp64=fp64, methods=getattr(st.MethodFlags, methods), forward=True)
    m.init()
    assert m.forwarding()
    u = _gather(m)
    for _ in range(3):
        m.step()
        u = jacobi_step_reference(u)
        m.synchronize()
        assert torch.equal(_gather(m), u)
        assert _check_halos(m, u, _FACES) == 0


@pytest.mark.parametrize("gpus", [[0], [0, 0, 0]])
def test_astaroth_forwarding_26dirs(st, gpus):
    """radius 3 in all 26 directions: edge and corner halos are forwarded too."""
    L = (48, 36, 30)
    m = st.AstarothSim(L, quantities=2, gpus=gpus, forward=True)
    m.init()
    assert m.forwarding()
    u = _gather(m)
    for _ in range(2):
        m.step()
        u = astaroth_step_reference(u)
    m.synchronize()
    assert torch.equal(_gather(m), u)
    assert _check_halos(m, u, _ALL26) == 0


@pytest.mark.parametrize("size", [(32, 32, 32), (67, 45, 33), (130, 64, 40)])
@pytest.mark.parametrize("gpus", [[0], [0, 0], [0, 0, 0, 0]])
@pytest.mark.parametrize("fp64", [False, True])
@pytest.mark.parametrize("sched", [1, 0])
def test_jacobi_temporal2_matches_oracle(st, size, gpus, fp64, sched):
    """Temporal blocking (stencil7x2: S o S per sweep, one depth-2 exchange per pair) is bitwise equal to single
    steps; run(5) = two fused pairs + one single step, run(16) = one captured graph block (single sub-domain).
    sched = work split: 1 = balanced segments, 0 = fixed z-chunks."""
    t = st.StencilTune()
    t.x2sched = sched
    m = st.Jacobi3D(size, gpus=gpus, fp64=fp64, temporal=2, tune=t)
    m.init()
    assert m.temporal_blocking()
    u = _gather(m)
    for n in (5, 16):
        m.run(n)
        for _ in range(n):
            u = jacobi_step_reference(u)
        m.synchronize()
        assert torch.equal(_gather(m), u), f"after run({n})"


@pytest.mark.parametrize("size,fp64", [((64, 40, 36), False), ((67, 45, 33), False), ((34, 30, 28), True),
                                       ((8, 12, 10), False), ((260, 64, 60), False), ((264, 64, 60), False),
                                       ((130, 40, 36), True)])
@pytest.mark.parametrize("gpus", [[0], [0, 0], [0, 0, 0, 0]])
@pytest.mark.parametrize("kind", ["jacobi", "astaroth"])
def test_temporal2_in_kernel_wrap(st, size, fp64, gpus, kind):
    """Fused pairs with in-kernel periodic wrap along the axes the decomposition leaves whole (the pair's exchange
    skips those self copies): bitwise equal to single steps, and to the same model with wrap_self=False. x wraps only
    for whole 16-B chunks (64, 8 fp32 and 34 fp64 do, 67 does not); run(5) ends on a single step, which refreshes
    every halo with the full exchange."""
    from stencil2_amd.ops import astaroth_step_reference
    cls, ref, kw = ((st.Jacobi3D, jacobi_step_reference, {}) if kind == "jacobi"
                    else (st.AstarothSim, astaroth_step_reference, {"quantities": 2}))
    ms = [cls(size, gpus=gpus, fp64=fp64, temporal=2, wrap_self=w, **kw) for w in (True, False)]
    for m in ms:
        m.init()
        assert m.temporal_blocking()
    pd = ms[0].domain.placement_dim()
    whole = sum(1 << a for a, n in enumerate((pd.x, pd.y, pd.z)) if n == 1)
    assert ms[1].wrap_axes() == 0
    assert ms[0].wrap_axes() & ~whole == 0 and ms[0].wrap_axes() & 6 == whole & 6
    V = 2 if fp64 else 4
    assert ms[0].wrap_axes() & 1 == (whole & 1 if size[0] % V == 0 and (size[0] // V) % 64 != 1 else 0)
    u = _gather(ms[0])
    for n in (5, 16, 2):
        for m in ms:
            m.run(n)
        for _ in range(n):
            u = ref(u)
        for m in ms:
            m.synchronize()
            assert torch.equal(_gather(m), u), f"wrap_axes={m.wrap_axes()} after run({n})"


@pytest.mark.parametrize("sched,scale", [(0, 1.0), (1, 1.0), (1, 1e-33)])
@pytest.mark.parametrize("kind,size", [("jacobi", (512, 120, 116)), ("jacobi", (512, 128, 120)),
                                       ("jacobi", (512, 512, 112)), ("astaroth", (512, 36, 28)),
                                       ("astaroth", (512, 13, 17)), ("astaroth", (512, 3, 16))])
def test_temporal3_matches_three_single_steps(st, kind, size, sched, scale):
    """Fused triples (stencil7x3_wrap_kernel, temporal=3, one GPU, every axis wrapped in-kernel): S(S(S(u))) bitwise
    equal to three single steps of the torch oracle; run(n) covers whole hipGraph blocks (18 steps), triples and the
    pair / single-step remainders; y extents that are not a multiple of the block's 6 output rows and a 3-row grid
    (every block row wraps onto itself twice). scale 1e-33 puts every sum below 2^-100, where the quotient is the
    true division."""
    from stencil2_amd.ops import astaroth_step_reference
    cls, ref, kw = ((st.Jacobi3D, jacobi_step_reference, {}) if kind == "jacobi"
                    else (st.AstarothSim, astaroth_step_reference, {"quantities": 2}))
    t = st.StencilTune()
    t.x3sched = sched
    m = cls(size, gpus=[0], temporal=3, tune=t, **kw)
    m.init()
    assert m.temporal_triples() and m.wrap_axes() == 7
    m.prepare()
    u = torch.rand((size[2], size[1], size[0]), device="cuda", generator=torch.Generator(device="cuda").manual_seed(5))
    u = u * scale
    for q in range(kw.get("quantities", 1)):
        m.interior(0, q).copy_(u)
    torch.cuda.synchronize()
    for n in (3, 7, 2, 20, 1):
        m.run(n)
        for _ in range(n):
            u = ref(u)
        m.synchronize()
        for q in range(kw.get("quantities", 1)):
            got = m.interior(0, q)
            bad = int((got != u).sum())
            assert bad == 0, f"run({n}) q{q}: {bad} cells differ, max {(got - u).abs().max().item()}"


def _set_field(m, u, quantities=1):
    for di in range(m.domain.num_domains()):
        d = m.domain.domain(di)
        o, s = d.origin(), d.size()
        for q in range(quantities):
            m.interior(di, q).copy_(u[o.z:o.z + s.z, o.y:o.y + s.y, o.x:o.x + s.x].to(m.interior(di, q).dtype))
    torch.cuda.synchronize()


# x cut by cost (1, 4, 4); (100, 3, 2) / (100, 2, 3) keep x whole
@pytest.mark.parametrize("kind,size,fp64,gpus,cost,scale", [
    ("jacobi", (512, 120, 116), False, [0], None, 1.0), ("jacobi", (1024, 240, 232), False, [0], None, 1.0),
    ("astaroth", (512, 36, 28), False, [0], None, 1.0), ("astaroth", (1536, 13, 17), False, [0], None, 1.0),
    ("astaroth", (512, 3, 16), False, [0], None, 1e-33), ("jacobi", (512, 120, 116), False, [0], None, 1e-33),
    ("jacobi", (256, 64, 64), True, [0], None, 1.0), ("astaroth", (512, 20, 24), True, [0], None, 1.0),
    ("astaroth", (256, 12, 16), True, [0], None, 1e-300),
    ("jacobi", (1024, 240, 232), False, [0, 0], (1, 4, 4), 1.0), ("astaroth", (2048, 30, 20), False, [0, 0, 0, 0], (1, 4, 4), 1.0),
    ("astaroth", (512, 40, 64), False, [0, 0, 0, 0], (100, 3, 2), 1.0), ("jacobi", (512, 240, 232), False, [0, 0], (100, 2, 3), 1.0),
    ("astaroth", (512, 24, 40), True, [0, 0], (1, 4, 4), 1.0)])
def test_temporal3_x_halos(st, kind, size, fp64, gpus, cost, scale):
    """Fused triples reading x from 3-deep halos (stencil7x3 XH form: 512-cell fp32 / 256-cell fp64 columns, the 3
    cells beyond each column end loaded per lane half, u1 / u2 computed on the column-end cells): every halo copied
    each triple (wrap_self=False: BASELINE config 2 as defined, one depth-3 exchange per three steps), on one
    sub-domain and on 2 / 4 sub-domains of one GPU with x, y or z cut; 1-3 columns per row; fp64; tiny sums (true
    division). Bitwise equal to single steps of the torch oracle, through graph blocks, triples and remainders."""
    from stencil2_amd.ops import astaroth_step_reference
    cls, ref, kw = ((st.Jacobi3D, jacobi_step_reference, {}) if kind == "jacobi"
                    else (st.AstarothSim, astaroth_step_reference, {"quantities": 2}))
    if cost is not None:
        kw["axis_cost"] = cost
    m = cls(size, gpus=gpus, temporal=3, fp64=fp64, wrap_self=False, **kw)
    m.init()
    assert m.temporal_triples() and m.wrap_axes() == 0, f"triples {m.temporal_triples()} wrap {m.wrap_axes()}"
    m.prepare()
    dt = torch.float64 if fp64 else torch.float32
    u = torch.rand((size[2], size[1], size[0]), device="cuda", dtype=dt,
                   generator=torch.Generator(device="cuda").manual_seed(7)) * scale
    nq = kw.get("quantities", 1)
    _set_field(m, u, nq)
    for n in (3, 7, 2, 20, 1):
        m.run(n)
        for _ in range(n):
            u = ref(u)
        m.synchronize()
        for q in range(nq):
            got = _gather(m, q).to(u.device)
            bad = int((got != u).sum())
            assert bad == 0, f"run({n}) q{q}: {bad} cells differ, max {(got - u).abs().max().item()}"


@pytest.mark.parametrize("kind,size,fp64", [("astaroth", (1024, 36, 28), False), ("jacobi", (1024, 240, 232), False),
                                            ("astaroth", (512, 20, 24), True), ("jacobi", (512, 120, 116), True)])
def test_temporal3_x_halos_where_x_cannot_wrap(st, kind, size, fp64):
    """One GPU, wrap_self=True, rows the whole-row triple cannot wrap (1024 fp32 cells, fp64): the model keeps fused
    triples by reading x from halos (the x self copies stay in the depth-3 exchange) and wraps only y and z; bitwise
    equal to single steps of the torch oracle."""
    from stencil2_amd.ops import astaroth_step_reference
    cls, ref, kw = ((st.Jacobi3D, jacobi_step_reference, {}) if kind == "jacobi"
                    else (st.AstarothSim, astaroth_step_reference, {"quantities": 1}))
    m = cls(size, gpus=[0], temporal=3, fp64=fp64, **kw)
    m.init()
    assert m.temporal_triples() and m.wrap_axes() == 6, f"triples {m.temporal_triples()} wrap {m.wrap_axes()}"
    dt = torch.float64 if fp64 else torch.float32
    u = torch.rand((size[2], size[1], size[0]), device="cuda", dtype=dt, generator=torch.Generator(device="cuda").manual_seed(9))
    _set_field(m, u)
    for n in (3, 20, 4):
        m.run(n)
        for _ in range(n):
            u = ref(u)
        m.synchronize()
        got = _gather(m).to(u.device)
        assert torch.equal(got, u), f"run({n}): {int((got != u).sum())} cells differ"


def test_temporal3_field_beyond_4gib(st):
    """A 1024 x 1024 x 1040 fp32 field (4.4 GB per buffer): the triple's buffer loads address one plane at a time
    (resource base per plane), so fields past 4 GiB (config 5: 1024^3 fp64, 8.6 GB per quantity) keep the triples"""
    from stencil2_amd.ops import astaroth_step_reference
    size = (1024, 1024, 1040)
    m = st.AstarothSim(size, quantities=1, gpus=[0], temporal=3)
    m.init()
    assert m.temporal_triples() and m.domain.domain(0).buffer_bytes(0) > (1 << 32)
    u = torch.rand((size[2], size[1], size[0]), device="cuda", generator=torch.Generator(device="cuda").manual_seed(2))
    _set_field(m, u)
    m.run(3)
    m.run(1)
    m.synchronize()
    for _ in range(4):
        u = astaroth_step_reference(u)
    got = m.interior(0)
    assert torch.equal(got, u), f"{int((got != u).sum())} cells differ"
    del m


# cuts follow the interface cost (NodePartition): 4*Y*Z for an x cut against 2*X*Z (y, cost 4,2,3) / 2*X*Y (z, 4,3,2)
@pytest.mark.parametrize("kind,size,gpus,cost", [("astaroth", (512, 300, 24), [0, 0], (4, 2, 3)),
                                                 ("astaroth", (512, 16, 300), [0, 0], (4, 3, 2)),
                                                 ("jacobi", (512, 300, 128), [0, 0], (4, 2, 3)),
                                                 ("astaroth", (512, 600, 24), [0, 0, 0, 0], (4, 2, 3))])
def test_temporal3_halo_axes(st, kind, size, gpus, cost):
    """Fused triples on sub-domains cut along y and/or z (several on one GPU, same-GPU depth-3 exchange): x wraps
    in-kernel, the cut axes read their 3-deep halos. Bitwise equal to single steps of the torch oracle."""
    from stencil2_amd.ops import astaroth_step_reference
    cls, ref, kw = ((st.Jacobi3D, jacobi_step_reference, {}) if kind == "jacobi"
                    else (st.AstarothSim, astaroth_step_reference, {"quantities": 2}))
    m = cls(size, gpus=gpus, temporal=3, axis_cost=cost, **kw)
    m.init()
    assert m.temporal_triples() and (m.wrap_axes() & 1) and m.wrap_axes() != 7, f"wrap_axes={m.wrap_axes()}"
    u = _gather(m)
    for n in (3, 7, 9, 2):
        m.run(n)
        for _ in range(n):
            u = ref(u)
        m.synchronize()
        assert torch.equal(_gather(m), u), f"run({n}) wrap_axes={m.wrap_axes()}"


@pytest.mark.parametrize("kind,size,gpus", [
    ("jacobi", (512, 120, 116), [0]), ("jacobi", (512, 300, 112), [0, 0]), ("astaroth", (512, 36, 28), [0]),
    ("astaroth", (512, 520, 40), [0, 0, 0, 0]),
    # ragged periodic rows: 2 / 3 / 4 chunks per lane, the row-end cells broadcast for the wrap
    ("astaroth", (645, 20, 24), [0]), ("astaroth", (301, 24, 20), [0]), ("astaroth", (300, 20, 16), [0]),
    ("astaroth", (768, 12, 16), [0]), ("astaroth", (646, 520, 12), [0, 0]), ("jacobi", (645, 136, 136), [0]),
    # tail rows: 3 chunks + one cell per lane (769-832 cells; the 4-GPU ladder's 813)
    ("astaroth", (813, 20, 24), [0]), ("astaroth", (769, 12, 16), [0]), ("astaroth", (832, 12, 16), [0]),
    ("astaroth", (800, 520, 12), [0, 0]), ("jacobi", (813, 168, 176), [0]), ("jacobi", (813, 432, 176), [0, 0]),
])
def test_temporal2_whole_row_kernel(st, kind, size, gpus):
    """Fused pairs on periodic rows of 257-832 cells take the whole-row kernel (one wave per row, x-neighbours by
    lane rotates, StencilTune.x2row; ragged rows broadcast their end cells, rows of 769-832 add one tail cell per
    lane): bitwise equal to single steps, with the
    hot/cold spheres (Jacobi) inside the grid, and to the column kernel (x2row = 0, which copies ragged x halos)."""
    from stencil2_amd.ops import astaroth_step_reference
    cls, ref, kw = ((st.Jacobi3D, jacobi_step_reference, {}) if kind == "jacobi"
                    else (st.AstarothSim, astaroth_step_reference, {"quantities": 2}))
    ms = []
    row = 1
    for r, early in ((row, False), (0, False), (row, True)):  # x2early: src / u1 rows published right after u1
        t = st.StencilTune()
        t.x2row = r
        t.x2early = early
        ms.append(cls(size, gpus=gpus, temporal=2, tune=t, axis_cost=(4, 2, 3), **kw))  # bench.py's cut: x stays whole
    for m in ms:
        m.init()
        assert m.temporal_blocking()
    assert ms[0].wrap_axes() & 1 and bool(ms[1].wrap_axes() & 1) == (size[0] % 4 == 0)
    u = _gather(ms[0])
    for n in (5, 16):
        for m in ms:
            m.run(n)
        for _ in range(n):
            u = ref(u)
        for m in ms:
            m.synchronize()
            assert torch.equal(_gather(m), u), f"model {ms.index(m)} (x2row, x2early = {row}/0/{row}+early) after run({n})"


@pytest.mark.parametrize("kind,size,gpus,fp64", [("jacobi", (512, 120, 116), [0], False),
                                                 ("jacobi", (200, 72, 64), [0, 0], False),
                                                 ("jacobi", (130, 40, 36), [0], False),
                                                 ("astaroth", (512, 36, 28), [0], False),
                                                 ("astaroth", (96, 260, 40), [0, 0, 0, 0], False),
                                                 ("astaroth", (66, 30, 20), [0, 0], True)])
def test_single_step_in_kernel_wrap(st, kind, size, gpus, fp64):
    """Single steps read the periodic image along every self-periodic axis in-kernel (StencilTune.wrap on the LDS
    kernel) and leave those self copies out of the exchange: bitwise equal to the torch oracle (spheres inside the
    grid for Jacobi) and to the model that copies every halo (wrap_self=False), through run() (hipGraph blocks) and
    step(); fp32 and fp64, x extents a multiple of the 16-B chunk or not."""
    from stencil2_amd.ops import astaroth_step_reference
    cls, ref, kw = ((st.Jacobi3D, jacobi_step_reference, {}) if kind == "jacobi"
                    else (st.AstarothSim, astaroth_step_reference, {"quantities": 2}))
    ms = [cls(size, gpus=gpus, temporal=1, wrap_self=ws, fp64=fp64, axis_cost=(4, 2, 3), **kw) for ws in (True, False)]
    for m in ms:
        m.init()
        assert not m.temporal_blocking()
    w = ms[0].domain.self_wrap_axes()
    v = 2 if fp64 else 4
    expect = w if size[0] % v == 0 else w & 6
    assert ms[0].step_wrap_axes() == expect and ms[1].step_wrap_axes() == 0
    assert (w == 7) == (len(gpus) == 1)
    u = _gather(ms[0])
    for n in (3, 16):
        for m in ms:
            m.run(n)
            m.step()
        for _ in range(n + 1):
            u = ref(u)
        for m in ms:
            m.synchronize()
            assert torch.equal(_gather(m), u), f"wrap_self={ms.index(m) == 0} after run({n}) + step()"


@pytest.mark.parametrize("kind,size,gpus,wrap,cost,fp64", [
    ("astaroth", (1024, 24, 20), [0], True, (4, 2, 3), False),     # periodic x: two 512-cell columns
    ("astaroth", (1024, 20, 16), [0], False, (4, 2, 3), False),    # x halos in memory
    ("astaroth", (512, 20, 24), [0], False, (4, 2, 3), False),     # one column between halos
    ("astaroth", (1024, 16, 20), [0, 0], True, (1, 1, 1), False),  # x cut: 512-wide halves, halos from the other half
    ("jacobi", (1024, 216, 212), [0], True, (4, 2, 3), False),     # spheres
    ("jacobi", (512, 120, 116), [0], False, (4, 2, 3), False),
    # fp64: 256-cell columns (two 2-double chunks per lane)
    ("astaroth", (1024, 24, 20), [0], True, (4, 2, 3), True),      # four periodic columns
    ("astaroth", (256, 20, 24), [0], True, (4, 2, 3), True),       # one column, wrapped onto itself
    ("astaroth", (512, 20, 16), [0], False, (4, 2, 3), True),      # x halos in memory
    ("astaroth", (512, 16, 20), [0, 0], True, (1, 1, 1), True),    # x cut: 256-wide halves
    ("jacobi", (1024, 216, 212), [0], True, (4, 2, 3), True),      # spheres
    ("jacobi", (256, 120, 116), [0], False, (4, 2, 3), True),
])
def test_temporal2_col512_kernel(st, kind, size, gpus, wrap, cost, fp64):
    """Fused pairs on x extents of whole two-chunk columns (512 fp32 / 256 fp64 cells) take the two-chunk column
    kernel (two chunks per lane, the column-end pairs by broadcast loads, stencil7x2_col2_kernel): bitwise equal to
    single steps and to the one-chunk column kernel (x2row = 0)."""
    from stencil2_amd.ops import astaroth_step_reference
    cls, ref, kw = ((st.Jacobi3D, jacobi_step_reference, {}) if kind == "jacobi"
                    else (st.AstarothSim, astaroth_step_reference, {"quantities": 2}))
    ms = []
    for row, early in ((1, False), (0, False), (1, True)):
        t = st.StencilTune()
        t.x2row = row
        t.x2early = early
        ms.append(cls(size, gpus=gpus, temporal=2, tune=t, wrap_self=wrap, axis_cost=cost, fp64=fp64, **kw))
    for m in ms:
        m.init()
        assert m.temporal_blocking()
    u = _gather(ms[0])
    for n in (5, 16):
        for m in ms:
            m.run(n)
        for _ in range(n):
            u = ref(u)
        for m in ms:
            m.synchronize()
            assert torch.equal(_gather(m), u), f"model {ms.index(m)} (col2 / column / col2 + x2early) after run({n})"


@pytest.mark.parametrize("temporal", [1, 2])
def test_prepare_graph_blocks(st, temporal):
    """prepare() records run()'s hipGraph blocks for both buffer parities without running anything: the field is
    unchanged by it, and later runs of either parity (odd step counts in between) match the oracle."""
    m = st.Jacobi3D((48, 40, 36), gpus=[0], temporal=temporal)
    m.init()
    u = _gather(m)
    m.prepare()
    m.synchronize()
    assert torch.equal(_gather(m), u)
    for n in (16, 3, 16, 1, 32):
        m.run(n)
        for _ in range(n):
            u = jacobi_step_reference(u)
    m.synchronize()
    assert torch.equal(_gather(m), u)


@pytest.mark.parametrize("temporal,size", [(1, (48, 40, 36)), (2, (48, 40, 36)), (3, (512, 120, 116))])
def test_prepare_whole_run_graphs(st, temporal, size):
    """prepare(runs) also records one graph per listed run length and parity (blocks plus remainder sweeps): nothing
    runs while recording, and run(n) replaying it from either parity (odd counts in between) matches the oracle."""
    m = st.Jacobi3D(size, gpus=[0], temporal=temporal)
    m.init()
    if temporal == 3:
        assert m.temporal_triples()
    u = _gather(m)
    m.prepare([20, 7, 1])
    m.synchronize()
    assert torch.equal(_gather(m), u)
    for n in (20, 7, 20, 1, 20, 5):
        m.run(n)
        for _ in range(n):
            u = jacobi_step_reference(u)
    m.synchronize()
    assert torch.equal(_gather(m), u)


def test_set_triple_schedule_keeps_results(st):
    """set_triple_schedule (bench.py's schedule choice) drops the recorded graphs and re-plans the lockstep launch:
    every schedule (sphere weight, leftover plan, parts) stays bitwise equal to the oracle across switches."""
    m = st.Jacobi3D((512, 120, 116), gpus=[0], temporal=3)
    m.init()
    assert m.temporal_triples()
    u = _gather(m)
    m.prepare([18])
    for sphw, left, parts in ((0.45, 3, 0), (0.3, 1, 0), (0.6, 2, 4), (0.0, 0, 3), (0.45, 2, 0)):
        m.set_triple_schedule(sphw, left, parts)
        m.prepare([18])
        for n in (18, 5):
            m.run(n)
            for _ in range(n):
                u = jacobi_step_reference(u)
    m.synchronize()
    assert torch.equal(_gather(m), u)


def test_temporal2_spheres_at_periodic_face_fall_back(st):
    """Spheres that reach a periodic face (radius x/10 on a thin y/z grid) make the fused pair's halo-ring step
    differ from the neighbour's: the model runs single steps there, still equal to the oracle."""
    m = st.Jacobi3D((260, 20, 18), gpus=[0], temporal=2)
    m.init()
    assert not m.temporal_blocking()
    u = _gather(m)
    m.run(4)
    for _ in range(4):
        u = jacobi_step_reference(u)
    m.synchronize()
    assert torch.equal(_gather(m), u)


@pytest.mark.parametrize("size", [(32, 32, 32), (67, 45, 33), (130, 70, 20)])
@pytest.mark.parametrize("gpus", [[0], [0, 0]])
def test_jacobi_mfma_variant_matches_oracle(st, size, gpus):
    """The matrix-core x-line update (StencilTune.variant = 8) is bitwise equal to the torch oracle: the banded
    16x16x4 fp32 MFMA sums exactly two exact products per output (a single rounding of vpx + vmx)."""
    t = st.StencilTune()
    t.variant = 8
    m = st.Jacobi3D(size, gpus=gpus, temporal=1, tune=t)
    m.init()
    u = _gather(m)
    m.run(3)
    for _ in range(3):
        u = jacobi_step_reference(u)
    m.synchronize()
    assert torch.equal(_gather(m), u)


def test_jacobi_mfma_variant_special_values(st):
    """signed zeros, tiny and subnormal values through the MFMA band product (finite inputs)"""
    t = st.StencilTune()
    t.variant = 8
    m = st.Jacobi3D((72, 20, 18), gpus=[0], temporal=1, tune=t)
    m.init()
    g = torch.Generator().manual_seed(3)
    pool = torch.tensor([0.0, -0.0, 1e-35, -1e-35, 3e-39, -3e-39, 1e-45, 0.5, -0.25, 7.0], dtype=torch.float32)
    it = m.interior(0)
    vals = pool[torch.randint(0, len(pool), tuple(it.shape), generator=g)]
    vals[3:6] = -0.0
    it.copy_(vals.to(it.device))
    torch.cuda.synchronize()
    u = _gather(m)
    m.run(2)
    for _ in range(2):
        u = jacobi_step_reference(u)
    m.synchronize()
    got = _gather(m)
    assert torch.equal(got.view(torch.int32), u.view(torch.int32)), int((got.view(torch.int32) != u.view(torch.int32)).sum())


@pytest.mark.parametrize("temporal,size", [(1, (72, 20, 18)), (2, (72, 20, 18)), (2, (512, 20, 18))])
@pytest.mark.parametrize("kind", ["jacobi", "astaroth"])
def test_stencil_special_values_bitwise(st, temporal, size, kind):
    """Fields with signed zeros, values below 2^-100 (the exact-/6 slow path), subnormals and mixed signs: the packed
    fp32 sums and the FMA division must stay bitwise equal to the torch oracle (0-started sums, IEEE division).
    512-cell rows: the whole-row fused kernel (Jacobi there falls back to single steps: its spheres reach the faces)."""
    from stencil2_amd.ops import astaroth_step_reference
    if kind == "jacobi":
        m = st.Jacobi3D(size, gpus=[0, 0], temporal=temporal)
        ref = jacobi_step_reference
    else:
        m = st.AstarothSim(size, quantities=1, gpus=[0, 0], temporal=temporal)
        ref = astaroth_step_reference
    m.init()
    g = torch.Generator().manual_seed(7)
    pool = torch.tensor([0.0, -0.0, 1e-35, -1e-35, 3e-39, -3e-39, 1e-45, 0.5, -0.25, 7.0], dtype=torch.float32)
    dd = m.domain
    for di in range(dd.num_domains()):
        it = m.interior(di)
        idx = torch.randint(0, len(pool), tuple(it.shape), generator=g)
        vals = pool[idx] * torch.where(torch.rand(tuple(it.shape), generator=g) < 0.3,
                                       torch.rand(tuple(it.shape), generator=g), torch.ones(()))
        # whole planes of zeros and of tiny values, so some six-neighbour sums are exactly +-0 or tiny
        vals[3:6] = -0.0
        vals[8:10] = 2e-36
        it.copy_(vals.to(it.device))
    torch.cuda.synchronize()
    u = _gather(m)
    m.run(4)
    for _ in range(4):
        u = ref(u)
    m.synchronize()
    got = _gather(m)
    assert torch.equal(got.view(torch.int32), u.view(torch.int32)), int((got.view(torch.int32) != u.view(torch.int32)).sum())


@pytest.mark.parametrize("methods", ["All", "Rccl", "Staged"])
@pytest.mark.parametrize("size,gpus", [((40, 36, 44), [0, 0]), ((67, 45, 33), [0, 0, 0, 0]), ((30, 28, 26), [0])])
@pytest.mark.parametrize("kind", ["jacobi", "astaroth"])
def test_temporal2_overlapped(st, methods, size, gpus, kind):
    """Overlapped fused pairs: S o S of the interior during the depth-2 exchange, the exterior slabs (thread per
    cell, stencil7x2_regions_kernel) after it -- bitwise equal to single steps."""
    from stencil2_amd.ops import astaroth_step_reference
    cls, ref, kw = ((st.Jacobi3D, jacobi_step_reference, {}) if kind == "jacobi"
                    else (st.AstarothSim, astaroth_step_reference, {"quantities": 2}))
    m = cls(size, gpus=gpus, methods=getattr(st.MethodFlags, methods), temporal=2, overlap=True,
            auto_overlap=False, **kw)
    m.init()
    assert m.temporal_blocking() and m.overlapping()
    u = _gather(m)
    m.run(7)  # three overlapped pairs and one single (overlapped) step
    for _ in range(7):
        u = ref(u)
    m.synchronize()
    assert torch.equal(_gather(m), u)


@pytest.mark.parametrize("zrow,mode", [("1", "1"), ("0", "1"), ("1", "2")])
@pytest.mark.parametrize("size,gpus,fake,kind", [((512, 112, 120), [0], 4, "jacobi"),
                                                 ((512, 112, 120), [0, 0], 4, "jacobi"),
                                                 ((512, 112, 120), [0, 0, 0, 0], 6, "jacobi"),
                                                 ((512, 20, 26), [0, 0], 6, "astaroth"),
                                                 ((645, 132, 136), [0, 0], 4, "jacobi")])
def test_temporal2_overlapped_zslab_row_kernel(st, zrow, mode, size, gpus, fake, kind):
    """Overlapped fused pairs with periodic 512-cell (and ragged) rows whose z (and y) faces are treated as remote
    (TransportOptions.fake_remote_axes: the multi-GPU split on one GPU): the z slabs go through the whole-row kernel
    with the slab as its z chunk (StencilTune.zslab_row, default) or the thin kernel; both bitwise equal to single
    steps. mode 2: the slabs after the interior sweep."""
    from stencil2_amd.ops import astaroth_step_reference
    t = st.StencilTune()
    t.zslab_row = zrow == "1"
    tr = st.TransportOptions()
    tr.fake_remote_axes = fake
    cls, ref, kw = ((st.Jacobi3D, jacobi_step_reference, {}) if kind == "jacobi"
                    else (st.AstarothSim, astaroth_step_reference, {"quantities": 2}))
    m = cls(size, gpus=gpus, temporal=2, overlap=True, axis_cost=(64, 3, 2), tune=t, transport=tr,
            overlap_mode=int(mode), **kw)
    m.init()
    assert m.temporal_blocking() and m.overlapping() and m.wrap_axes() == (1 if fake == 6 else 3)
    assert m.domain.placement_dim().x == 1 and m.overlap_mode() == int(mode)
    u = _gather(m)
    m.run(6)
    for _ in range(6):
        u = ref(u)
    m.synchronize()
    assert torch.equal(_gather(m), u)


@pytest.mark.parametrize("fake,reserve,lockstep", [(None, 8, "1"), ("4", 8, "1"), ("4", 4, "1"), ("4", 8, "0"),
                                                    ("6", 8, "1")])
@pytest.mark.parametrize("alt", [False, True])
def test_temporal2_row_kernel_lockstep_quarters(st, fake, reserve, lockstep, alt):
    """Whole-row fused pairs over 64 row groups: the lockstep schedule (four blocks per column for the first
    blocks/4 columns, the rest as short second segments: 256 / 248 / 252 resident blocks) and the balanced one are
    bitwise equal to single steps (Astaroth proxy: no spheres, any grid thickness)."""
    from stencil2_amd.ops import astaroth_step_reference
    t = st.StencilTune()
    t.x2lockstep = lockstep == "1"
    t.x2reserve = reserve
    t.alternate_z = alt  # per-pair z-direction flip (on by default since r4)
    tr = st.TransportOptions()
    tr.fake_remote_axes = int(fake or 0)
    m = st.AstarothSim((512, 512, 72), quantities=1, gpus=[0], temporal=2, tune=t, axis_cost=(64, 3, 2),
                       transport=tr)
    m.init()
    assert m.temporal_blocking() and m.overlapping() == bool(fake)
    u = _gather(m)
    m.run(4)
    for _ in range(4):
        u = astaroth_step_reference(u)
    m.synchronize()
    assert torch.equal(_gather(m), u)


@pytest.mark.parametrize("size,fp64", [((512, 320, 112), False), ((645, 200, 160), False), ((813, 136, 256), False),
                                       ((1024, 128, 128), False),
                                       # 70 row groups: 2 rounds x 35 groups x 7 parts
                                       ((512, 560, 112), False),
                                       # 81 row groups: quarters over 64 + 17 leftover groups as second segments
                                       ((512, 648, 240), False),
                                       # more row groups than blocks: rounds of whole columns (seg 3)
                                       ((512, 2112, 16), False), ((2048, 1040, 16), False), ((1024, 1040, 16), True)])
def test_temporal2_row_kernel_lockstep_parts(st, size, fp64):
    """Grids of fewer row groups than resident blocks / 4 run lockstep with P = blocks / columns z parts per column
    (40 columns: P = 6 over 240 blocks; 25 ragged 645-cell columns: P = 10; 17 tail-row columns: P = 15 over 255;
    the 512-cell column kernel over 2 x 16 columns: P = 8); grids of more row groups than blocks march rounds of
    whole columns (264 row groups: 2 rounds; 4 x 130 fp32 512-cell / fp64 256-cell columns: 3 rounds): bitwise equal
    to single steps."""
    from stencil2_amd.ops import astaroth_step_reference
    m = st.AstarothSim(size, quantities=1, gpus=[0], temporal=2, axis_cost=(64, 3, 2), fp64=fp64)
    m.init()
    assert m.temporal_blocking()
    u = _gather(m)
    for n in (2, 6):
        m.run(n)
        for _ in range(n):
            u = astaroth_step_reference(u)
        m.synchronize()
        assert torch.equal(_gather(m), u), f"after run({n})"


@pytest.mark.parametrize("methods", ["Rccl", "Staged", "PeerCopy", "PeerCopyEngine", "PeerCopyPeerApi"])
def test_jacobi_temporal2_transports(st, methods):
    """depth-2 exchanges (faces 2, edges 1) over every in-process transport, then fused pairs (PeerCopyEngine: the
    peer messages over DMA-engine copies, including the in-kernel-wrap subset prepared by prepare_skip_wrapped;
    PeerCopyPeerApi: those copies through hipMemcpyPeerAsync)"""
    tr = st.TransportOptions()
    if methods in ("PeerCopyEngine", "PeerCopyPeerApi"):
        tr.peer_copy = st.TransportOptions.Copy.Engine
        tr.peer_api_same_device = methods == "PeerCopyPeerApi"
        methods = "PeerCopy"
    m = st.Jacobi3D((40, 36, 44), gpus=[0, 0], methods=getattr(st.MethodFlags, methods), temporal=2, transport=tr)
    m.init()
    assert m.temporal_blocking()
    u = _gather(m)
    m.run(6)
    for _ in range(6):
        u = jacobi_step_reference(u)
    m.synchronize()
    assert torch.equal(_gather(m), u)


@pytest.mark.parametrize("gpus", [[0], [0, 0, 0]])
def test_astaroth_temporal2(st, gpus):
    L = (48, 36, 30)
    m = st.AstarothSim(L, quantities=2, gpus=gpus, temporal=2)
    m.init()
    assert m.temporal_blocking()
    u = _gather(m)
    m.run(4)
    for _ in range(4):
        u = astaroth_step_reference(u)
    m.synchronize()
    assert torch.equal(_gather(m), u)


def test_jacobi_fp64_device(st):
    m = st.Jacobi3D((40, 36, 20), gpus=[0], fp64=True)
    m.init()
    u = _gather(m)
    for _ in range(3):
        m.step()
        u = jacobi_step_reference(u)
    m.synchronize()
    assert torch.equal(_gather(m), u)


def test_astaroth_device_matches_oracle(st):
    L = (40, 34, 28)
    m = st.AstarothSim(L, quantities=2, gpus=[0, 0], forward=False)
    m.init()
    u = _gather(m)
    assert torch.allclose(u, astaroth_init_reference(L, 3, 10.0), atol=1e-6)
    for _ in range(3):
        m.step()
        u = astaroth_step_reference(u)
    m.synchronize()
    assert torch.equal(_gather(m), u)


@pytest.mark.parametrize("radius", ["r1", "fec", "asym"])
def test_colocated_ipc_two_ranks_one_gpu(radius):
    outs = run_ranks(2, WORKER, ["exchange", radius, "20,12,10"],
                     env_extra={"MP_DEVICE": "1", "MP_METHODS": "Colocated|Kernel", "STENCIL_WAIT_TIMEOUT": "20"})
    for rc, out in outs:
        assert rc == 0, out[-3000:]


@pytest.mark.parametrize("inbox,copy,completion,fuse", [("Uncached", "Engine", "Kernel", "1"),
                                                        ("Coarse", "Store", "Kernel", "1"),
                                                        ("Coarse", "Engine", "Kernel", "1"),
                                                        ("Fine", "Store", "Kernel", "1"),
                                                        ("Uncached", "Store", "Kernel", "0"),
                                                        ("Uncached", "Engine", "Kernel", "0"),
                                                        ("Uncached", "Store", "StreamOp", "1"),
                                                        ("Coarse", "Engine", "StreamOp", "1"),
                                                        ("Uncached", "Store", "IpcEvent", "1"),
                                                        ("Coarse", "Store", "IpcEvent", "1"),
                                                        ("Uncached", "Engine", "IpcEvent", "1")])
def test_colocated_transport_variants_two_ranks(inbox, copy, completion, fuse):
    """Every TransportOptions variant of the HIP IPC transport (receive-slot memory, kernel stores vs DMA-engine
    copies, flag waits/signals fused into the pack/unpack kernels or separate spin kernels, stream wait/write
    operations, or interprocess events with host notify/ack -- the reference's design): coordinate oracle over
    faces, edges and corners, then fused Jacobi pairs vs the torch oracle, two ranks sharing one GPU."""
    env = {"MP_DEVICE": "1", "MP_METHODS": "Colocated|Kernel", "STENCIL_WAIT_TIMEOUT": "20", "MP_INBOX": inbox,
           "MP_COLO_COPY": copy, "MP_COMPLETION": completion, "MP_FUSE_FLAGS": fuse}
    for rc, out in run_ranks(2, WORKER, ["exchange", "fec", "20,12,10"], env_extra=env):
        assert rc == 0, out[-3000:]
    env.update({"MP_METHODS": "All", "MP_TEMPORAL": "2", "MP_EXPECT_OVERLAP": "1"})
    for rc, out in run_ranks(2, WORKER, ["jacobi", "48,48,48"], env_extra=env):
        assert rc == 0, out[-3000:]
        assert "jacobi bad 0" in out


@pytest.mark.parametrize("ranks", [2, 3])
def test_ipc_event_handle_roundtrip(ranks):
    """reference test/test_cuda_mpi_cudaipc.cu:8-45: rank 0's interprocess event handle opens on every other rank,
    and their hipStreamWaitEvent on it holds their stream until rank 0's recorded work (a 0.2-s spin) is done"""
    outs = run_ranks(ranks, WORKER, ["ipcevent"], env_extra={"MP_DEVICE": "1"}, timeout=90)
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "'ok': True" in out, out[-2000:]


@pytest.mark.parametrize("completion,iters", [("Kernel", "4"), ("StreamOp", "4"), ("IpcEvent", "4"), ("Kernel", "24"),
                                              ("IpcEvent", "24")])
def test_colocated_caller_stream_two_ranks(completion, iters):
    """co-located exchanges blocking, stream-ordered on a caller (torch) stream and on the comm streams, each
    completion kind (bench.py's exchange loops), coordinate oracle; 24 per phase: over 100 event records"""
    outs = run_ranks(2, WORKER, ["streamloop", "64,48,80"],
                     env_extra={"MP_DEVICE": "1", "STENCIL_WAIT_TIMEOUT": "20", "MP_COMPLETION": completion,
                                "MP_ITERS": iters}, timeout=90)
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "streamloop bad 0" in out, out[-2000:]


def test_ipc_event_domains_in_sequence_and_host_run_ahead():
    """Acks drained at teardown (a second IpcEvent domain on the same group starts clean) and replaced
    interprocess events retired by device progress (48 stream-ordered exchanges behind a 1-s spin of the stream)"""
    outs = run_ranks(2, WORKER, ["ipcseq", "64,48,80"],
                     env_extra={"MP_DEVICE": "1", "STENCIL_WAIT_TIMEOUT": "20"}, timeout=100)
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "ipcseq bad 0" in out, out[-2000:]


def test_colocated_completion_switching_two_ranks():
    """set_completion between exchanges: interprocess events (realized with them) -> spin kernels -> events again
    (30 exchanges: past the event replacement) -> stream ops -> events -> kernels; coordinate oracle throughout"""
    outs = run_ranks(2, WORKER, ["streamloop", "64,48,80"],
                     env_extra={"MP_DEVICE": "1", "STENCIL_WAIT_TIMEOUT": "20", "MP_COMPLETION": "IpcEvent",
                                "MP_SWITCH": "1"}, timeout=120)
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "switch bad 0" in out, out[-2000:]


def test_rccl_init_failure_falls_back_to_staged(st):
    """An RCCL communicator that cannot be created (forced) turns every RCCL channel into a host-staged one
    (agreed on by all ranks) instead of aborting; the fused pairs stay exact."""
    tr = st.TransportOptions()
    tr.fail_rccl_init = True
    m = st.Jacobi3D((40, 36, 44), gpus=[0, 0], methods=st.MethodFlags.Rccl, temporal=2, transport=tr)
    m.init()
    dd = m.domain
    assert dd.exchange_bytes_for_method(st.MethodFlags.Rccl) == 0
    assert dd.exchange_bytes_for_method(st.MethodFlags.Staged) > 0
    u = _gather(m)
    m.run(4)
    for _ in range(4):
        u = jacobi_step_reference(u)
    m.synchronize()
    assert torch.equal(_gather(m), u)


def test_self_test_ladder_two_ranks():
    """DistributedDomain.set_self_test: the probe exchange passes with the co-located IPC transport (nothing dropped);
    with the IPC probe forced to fail, Colocated is dropped and the shared-GPU pairs are host-staged, still exact."""
    for fail in ("0", "1"):
        outs = run_ranks(2, WORKER, ["selftest", "48,40,36"],
                         env_extra={"MP_DEVICE": "1", "MP_METHODS": "All", "STENCIL_WAIT_TIMEOUT": "20",
                                    "MP_IPC_PROBE_FAIL": fail})
        for rc, out in outs:
            assert rc == 0, out[-3000:]
            assert "selftest bad 0" in out, out[-2000:]
            assert ("colo" in out.split("methods ")[-1].split()[0]) == (fail == "0"), out[-2000:]


@pytest.mark.parametrize("temporal,ranks", [("1", 2), ("2", 2), ("2", 4), ("2", 8)])
def test_colocated_ipc_jacobi_two_ranks(temporal, ranks):
    """Jacobi over HIP IPC between ranks sharing one GPU. Fused pairs overlap automatically here (the split axes
    are y/z): S o S of the local interior runs while the remote halos are in flight."""
    outs = run_ranks(ranks, WORKER, ["jacobi", "48,48,48"],  # a cube: cut along y, then z (8 ranks: 1x4x2)
                     env_extra={"MP_DEVICE": "1", "MP_METHODS": "All", "STENCIL_WAIT_TIMEOUT": "20",
                                "MP_TEMPORAL": temporal, "MP_EXPECT_OVERLAP": "1"})
    for rc, out in outs:
        assert rc == 0, out[-3000:]


def test_colocated_ipc_overlap_toggle_two_ranks():
    """Fused pairs over HIP IPC switched from overlapped to whole-region and back (StencilModel::set_overlap, the
    bench's warm-up choice): bitwise equal to the oracle throughout."""
    outs = run_ranks(2, WORKER, ["jacobi", "48,48,48"],
                     env_extra={"MP_DEVICE": "1", "MP_METHODS": "All", "STENCIL_WAIT_TIMEOUT": "20",
                                "MP_TEMPORAL": "2", "MP_EXPECT_OVERLAP": "1", "MP_TOGGLE_OVERLAP": "1"})
    for rc, out in outs:
        assert rc == 0, out[-3000:]


# cuts follow the interface cost (NodePartition): 4*Y*Z for an x cut against 2*X*Z (y, cost 4,2,3) / 2*X*Y (z, 4,3,2)
# modes 3 / 4 (pipelined) need every remote halo along z
@pytest.mark.parametrize("kind,size,cost,ranks,mode", [
    ("astaroth", "512,264,16", "4,2,3", 2, "0"), ("jacobi", "512,300,128", "4,2,3", 2, "0"),
    ("astaroth", "512,600,24", "4,2,3", 4, "0"),
    *[("astaroth", "512,16,300", "4,3,2", 2, md) for md in ("0", "4", "3")],
    ("jacobi", "512,192,600", "4,3,2", 2, "4"), ("astaroth", "512,16,600", "4,3,2", 4, "4")])
def test_triples_across_ranks(kind, size, cost, ranks, mode):
    """Fused triples with remote halos (multi-GPU layout rehearsed by ranks sharing one GPU over HIP IPC): x wrapped
    in-kernel, the cut axes read the 3-deep halos of one exchange per three steps. The overlapped pairs are the
    auto default; set_overlap_mode(0) (the bench's whole-region candidate) switches to triples, mode 4 to pipelined
    triples (each depth-3 exchange gated on the previous triple's published boundary planes), mode 3 to pipelined
    pairs publishing 3 planes per face. Bitwise vs the oracle through single steps, pairs and triples."""
    outs = run_ranks(ranks, WORKER, ["jacobi", size],
                     env_extra={"MP_DEVICE": "1", "MP_METHODS": "All", "STENCIL_WAIT_TIMEOUT": "20",
                                "MP_TEMPORAL": "3", "MP_KIND": kind, "MP_RANDOM": "1", "MP_AXIS_COST": cost,
                                "MP_TOGGLE_OVERLAP": "1", "MP_TOGGLE_MODES": mode, "MP_TOGGLE_STEPS": "10",
                                "MP_EXPECT_TRIPLES": "0" if mode == "3" else "1"})
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "jacobi bad 0" in out, out[-2000:]


@pytest.mark.parametrize("kind,size,ranks", [("astaroth", "1024,36,40", 2), ("jacobi", "1024,240,232", 2),
                                             ("astaroth", "2048,24,20", 4)])
def test_x_halo_triples_across_ranks(kind, size, ranks):
    """x cut between ranks sharing one GPU over HIP IPC (cost 1,4,4): the fused triples read x from the 3-deep halos
    another rank sends (XH columns, faces / edges / corners through one depth-3 exchange per three steps), y / z
    wrapped in-kernel. Bitwise vs the oracle through single steps and triples."""
    outs = run_ranks(ranks, WORKER, ["jacobi", size],
                     env_extra={"MP_DEVICE": "1", "MP_METHODS": "All", "STENCIL_WAIT_TIMEOUT": "20",
                                "MP_TEMPORAL": "3", "MP_KIND": kind, "MP_RANDOM": "1", "MP_AXIS_COST": "1,4,4",
                                "MP_RUN_STEPS": "9", "MP_EXPECT_TRIPLES": "1", "MP_EXPECT_WRAP": "6"})
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "jacobi bad 0" in out, out[-2000:]


@pytest.mark.parametrize("size,cost", [("512,264,16", "4,2,3"), ("1024,520,12", "4,2,3"), ("645,520,12", "4,2,3"),
                                       ("512,16,300", "4,3,2"), ("645,12,520", "4,3,2")])  # y cut / z cut
def test_colocated_ipc_wide_rows_two_ranks(size, cost):
    """The whole-row (512, ragged 645) and 512-cell column (1024) fused-pair kernels in the overlapped multi-rank
    step: y (cost 4,2,3) or z (the default 4,3,2) is cut between two ranks sharing one GPU (HIP IPC), x stays whole
    and wrapped in-kernel (also in the exterior slabs); S o S of the local interior runs while the remote halos are
    in flight (Astaroth proxy from an analytic field, bitwise vs the oracle)."""
    outs = run_ranks(2, WORKER, ["jacobi", size],
                     env_extra={"MP_DEVICE": "1", "MP_METHODS": "All", "STENCIL_WAIT_TIMEOUT": "20",
                                "MP_TEMPORAL": "2", "MP_KIND": "astaroth", "MP_EXPECT_OVERLAP": "1",
                                "MP_AXIS_COST": cost, "MP_EXPECT_WRAP": "5" if cost == "4,2,3" else "3"})
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "jacobi bad 0" in out


@pytest.mark.parametrize("kind,size,cost", [("astaroth", "512,16,300", "4,3,2"), ("jacobi", "96,80,36", "4,2,3"),
                                            ("astaroth", "645,12,520", "4,3,2")])
def test_colocated_single_steps_local_interior(kind, size, cost):
    """Overlapped single steps across two ranks sharing one GPU (HIP IPC): the interior is shrunk only at the remote
    faces (get_local_interior) and swept during the transfer, the self-periodic axes are wrapped in-kernel and left
    out of the exchange, the slabs at the remote faces follow (shell kernel with wrap). Bitwise vs the oracle."""
    expect = "3" if cost == "4,3,2" else "5"
    if size.startswith("645"):
        expect = "2"  # ragged x: single steps copy the x faces (whole 16-B chunks only)
    outs = run_ranks(2, WORKER, ["jacobi", size],
                     env_extra={"MP_DEVICE": "1", "MP_METHODS": "All", "STENCIL_WAIT_TIMEOUT": "20",
                                "MP_TEMPORAL": "1", "MP_KIND": kind, "MP_EXPECT_OVERLAP": "1",
                                "MP_AXIS_COST": cost, "MP_EXPECT_STEP_WRAP": expect})
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "jacobi bad 0" in out


def test_ipc_probe_failure_falls_back_on_shared_gpu():
    """Co-located ranks on one GPU whose IPC pre-flight fails (forced) must not pick RCCL (it refuses two ranks on
    one device): the runtime drops Colocated and Rccl and stages through the host; results stay exact."""
    outs = run_ranks(2, WORKER, ["jacobi", "48,48,48"],
                     env_extra={"MP_DEVICE": "1", "MP_METHODS": "All", "STENCIL_WAIT_TIMEOUT": "20",
                                "MP_TEMPORAL": "2", "MP_IPC_PROBE_FAIL": "1"})
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "jacobi bad 0" in out
        # only the pairs on the shared GPU are staged: here that is every cross-rank pair, none left on RCCL/IPC
        assert "bytes_Rccl=0 " in out and "bytes_Colocated=0 " in out and "bytes_Staged=0 " not in out, out[-2000:]


@pytest.mark.parametrize("methods,copy,fuse,completion", [("Colocated|Kernel", "Store", "1", "Kernel"),
                                                          ("Colocated|Kernel", "Store", "0", "Kernel"),
                                                          ("Colocated|Kernel", "Engine", "1", "Kernel"),
                                                          ("Colocated|Kernel", "Store", "1", "IpcEvent"),
                                                          ("Staged|Kernel", "Store", "1", "Kernel")])
def test_race_canary_two_ranks_one_gpu(methods, copy, fuse, completion):
    """Race canary over HIP IPC (double-buffered inboxes + credits; pack-kernel stores or DMA-engine copies) and the
    staged path, with jitter. Every host wait on a peer is bounded by STENCIL_WAIT_TIMEOUT and a stalled rank dumps
    its stacks (MP_STALL_DUMP_S), so a stall fails with every rank's phase instead of hanging."""
    outs = run_ranks(2, WORKER, ["canary", "fec", "20,12,10"],  # ~2.5 s normally; 90 s: rank outputs on a hang
                     env_extra={"MP_DEVICE": "1", "MP_METHODS": methods, "STENCIL_WAIT_TIMEOUT": "20",
                                "MP_JITTER_US": "200", "MP_COLO_COPY": copy, "MP_STALL_DUMP_S": "30",
                                "MP_FUSE_FLAGS": fuse, "MP_COMPLETION": completion}, timeout=90)
    for rc, out in outs:
        assert rc == 0, out[-3000:]


@pytest.mark.parametrize("methods", ["Rccl|Kernel", "Staged|Kernel"])
def test_jacobi_temporal2_two_ranks_other_transports(methods):
    """fused pairs over the staged transport, and over Rccl|Kernel between ranks that share one GPU: RCCL refuses a
    GPU driven by two ranks, so exactly those pairs (here: all cross-rank pairs) are host-staged"""
    outs = run_ranks(2, WORKER, ["jacobi", "36,20,24"],
                     env_extra={"MP_DEVICE": "1", "MP_METHODS": methods, "STENCIL_WAIT_TIMEOUT": "20", "MP_TEMPORAL": "2"})
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "jacobi bad 0" in out
        assert "bytes_Rccl=0 " in out and "bytes_Staged=0 " not in out, out[-2000:]


def test_staged_two_ranks_one_gpu():
    outs = run_ranks(2, WORKER, ["exchange", "r1", "16,12,10"], env_extra={"MP_DEVICE": "1", "MP_METHODS": "Staged|Kernel"})
    for rc, out in outs:
        assert rc == 0, out[-3000:]


@pytest.mark.parametrize("with_exchange", [False, True])
def test_headline_config_bitwise(st, with_exchange):
    """The driver's exact path: `bench.py --gpus 1 --steps 20 --warmup 5` builds this model (512^3 Jacobi3D fp32 on
    one GPU, temporal=3, bench.py's default StencilTune: lockstep triples with 0.3-weighted sphere parts, 128-B
    interiors, MaxLink decomposition), prepare()s the 18-step hipGraph blocks, runs 5 warm-up steps and times 20.
    with_exchange: the same with every halo copied each triple (wrap_self=False, shared halo lines: bench.py's
    extra.gcells_with_exchange model, BASELINE config 2 as defined, fused triples reading x from halos). From a
    random field, bitwise vs the torch oracle on GPU tensors (reference test style: test/test_exchange.cu:135-201)."""
    m = st.Jacobi3D((512, 512, 512), gpus=[0], temporal=3, tune=st.StencilTune(), axis_cost=(4, 3, 2),
                    partition=st.PartitionObjective.MaxLink, wrap_self=not with_exchange,
                    shared_halo_line=with_exchange)
    m.init()
    assert m.temporal_triples() and not m.overlapping()
    assert m.wrap_axes() == (0 if with_exchange else 7)
    m.prepare()
    u = torch.rand((512, 512, 512), device="cuda", generator=torch.Generator(device="cuda").manual_seed(3))
    m.interior(0).copy_(u)
    torch.cuda.synchronize()
    m.run(5)
    m.run(20)
    m.synchronize()
    for _ in range(25):
        u = jacobi_step_reference(u)
    got = m.interior(0)
    assert torch.equal(got, u), f"{int((got != u).sum())} cells differ"


@pytest.mark.parametrize("mode", ["0", "1", "2", "3", "3031"])
def test_headline_two_rank_exact_grid_bitwise(mode):
    """bench.py's 2-GPU weak-scaling grid (512x512x1024, cut 1x1x2, 512^3 per rank) with two ranks sharing one GPU
    over HIP IPC: fused pairs overlapped with the slabs beside (1) or after (2) the interior sweep, whole-region
    (0), or pipelined (3: each sweep publishes its boundary planes, the next pair's exchange is gated on them and
    runs beside the rest of the sweep), and switching 3 -> 0 -> 3 -> 1; from a random field, bitwise vs the torch
    oracle (computed on the GPU) after 1 + 8 + 16 steps."""
    outs = run_ranks(2, WORKER, ["jacobi", "512,512,1024"],
                     env_extra={"MP_DEVICE": "1", "MP_METHODS": "All", "STENCIL_WAIT_TIMEOUT": "30",
                                "MP_TEMPORAL": "2", "MP_RANDOM": "1", "MP_PREPARE": "1", "MP_SINGLE_STEPS": "1",
                                "MP_RUN_STEPS": "8", "MP_TOGGLE_OVERLAP": "1", "MP_TOGGLE_MODES": mode},
                     timeout=200)
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "jacobi bad 0" in out and "dim (1, 1, 2)" in out.replace("Dim3", ""), out[-2000:]
        assert f"overlap {mode[-1] != '0'}" in out, out[-2000:]


@pytest.mark.parametrize("mode", ["0", "4", "3", "1", "4304"])
def test_headline_two_rank_triples_bitwise(mode):
    """The same 2-GPU weak-scaling grid with temporal=3 (bench.py's default): depth-3 halos, whole-region fused
    triples (0), pipelined triples (4: each triple publishes its first / last 3 z planes early, the next depth-3
    exchange is gated on them), pipelined pairs publishing 3 planes (3), overlapped pairs (1), and switching
    4 -> 3 -> 0 -> 4; bitwise vs the torch oracle (on the GPU) after 1 + 8 + 16 steps."""
    outs = run_ranks(2, WORKER, ["jacobi", "512,512,1024"],
                     env_extra={"MP_DEVICE": "1", "MP_METHODS": "All", "STENCIL_WAIT_TIMEOUT": "30",
                                "MP_TEMPORAL": "3", "MP_RANDOM": "1", "MP_PREPARE": "1", "MP_SINGLE_STEPS": "1",
                                "MP_RUN_STEPS": "8", "MP_TOGGLE_OVERLAP": "1", "MP_TOGGLE_MODES": mode,
                                "MP_EXPECT_TRIPLES": "1" if mode[-1] in "04" else "0"},
                     timeout=200)
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "jacobi bad 0" in out and "dim (1, 1, 2)" in out.replace("Dim3", ""), out[-2000:]
        assert f"overlap {mode[-1] in '123'}" in out, out[-2000:]


def test_smoke_entry():
    import __graft_entry__ as g

    g.smoke()


def test_topology_links(st):
    """GPU topology (reference gpu_topology.cpp NVML distance): amd-smi when available, HIP link query otherwise."""
    from stencil2_amd import _C
    links = _C.gpu_links()
    n = st.device_count()
    assert len(links) == n * n
    for li in links:
        if li["src"] == li["dst"]:
            assert li["type"] == "self" and li["distance"] == pytest.approx(0.1)
        else:
            assert li["source"] in ("amd-smi", "hip", "none") and li["distance"] >= 0.5
    assert _C.gpu_numa_node(0) >= -1
    print("amd-smi:", _C.amdsmi_available(), "numa(0):", _C.gpu_numa_node(0))


@pytest.mark.parametrize("kind,size,fp64,gpus,temporal,wrap", [
    ("jacobi", (512, 120, 116), False, [0], 2, True),    # whole-row kernel, x wrapped in-kernel
    ("jacobi", (512, 20, 18), False, [0], 2, True),      # thin grid: spheres at the faces, single steps
    ("jacobi", (64, 36, 30), False, [0, 0], 2, True),    # column kernel (wrap lanes read left of raw x = 0)
    ("jacobi", (67, 36, 30), False, [0, 0], 2, True),    # ragged x: x faces copied
    ("jacobi", (64, 36, 30), True, [0, 0], 2, False),    # fp64, every halo copied
    ("jacobi", (48, 40, 36), False, [0, 0, 0], 1, True),  # single steps
    ("astaroth", (512, 16, 24), False, [0], 2, True),    # radius 3 (12-B x halos)
    ("astaroth", (40, 34, 28), True, [0, 0], 1, False)])  # radius 3 fp64 (24-B x halos)
def test_x_halo_aligned_layout_models(st, kind, size, fp64, gpus, temporal, wrap):
    """Halo-aligned x layout (LocalDomain.set_x_halo_align): the interior starts 16-B aligned inside its row's first
    64-B sector, the x halos share the interior's end sectors. The 16-B chunk kernels (whole-row, column, LDS single
    step) run on it unchanged: bitwise vs the torch oracle and vs the default layout."""
    from stencil2_amd.ops import astaroth_step_reference
    cls, ref, kw = ((st.Jacobi3D, jacobi_step_reference, {}) if kind == "jacobi"
                    else (st.AstarothSim, astaroth_step_reference, {"quantities": 2}))
    ms = [cls(size, gpus=gpus, fp64=fp64, temporal=temporal, wrap_self=wrap, x_halo_align=a, **kw)
          for a in (True, False)]
    for m in ms:
        m.init()
    d = ms[0].domain.domain(0)
    es = d.elem_size(0)
    first = d.curr_ptr(0) + d.radius().x(-1) * es
    assert first % 16 == 0 and first % 64 != 0 and d.x_halo_align()
    assert ms[0].temporal_blocking() == ms[1].temporal_blocking() == (temporal == 2 and size[2] > 20)
    assert ms[0].wrap_axes() == ms[1].wrap_axes() and ms[0].step_wrap_axes() == ms[1].step_wrap_axes()
    u = _gather(ms[0])
    for n in (5, 4):
        for m in ms:
            m.run(n)
        for _ in range(n):
            u = ref(u)
        for m in ms:
            m.synchronize()
        assert torch.equal(_gather(ms[0]), u)
        assert torch.equal(_gather(ms[1]), u)


@pytest.mark.parametrize("gpus,methods", [([0], "Kernel"), ([0, 0, 0], "Kernel"), ([0, 0], "PeerCopy"),
                                          ([0, 0], "Staged")])
@pytest.mark.parametrize("rname", ["r1", "fec", "asym"])
def test_x_halo_aligned_layout_exchange(st, gpus, methods, rname):
    radius = _radii(st)[rname]
    dd = st.DistributedDomain(19, 13, 11, group=st.make_single_group())
    dd.set_radius(radius)
    dd.set_gpus(gpus)
    dd.set_methods(getattr(st.MethodFlags, methods))
    dd.set_x_halo_align(True)
    q = dd.add_data("q", torch.int64)
    q2 = dd.add_data("f", torch.float32)
    dd.realize()
    for it in range(2):
        fill_coords(dd, q)
        fill_coords(dd, q2)
        dd.exchange()
        assert check_exchange(dd, q, radius) == 0 and check_exchange(dd, q2, radius) == 0
        dd.swap()


def test_x_halo_aligned_two_ranks_ipc():
    """the layout across ranks sharing one GPU (HIP IPC pack/unpack into the aligned halos), fused pairs bitwise"""
    outs = run_ranks(2, WORKER, ["jacobi", "512,120,232"],
                     env_extra={"MP_DEVICE": "1", "MP_METHODS": "All", "STENCIL_WAIT_TIMEOUT": "20",
                                "MP_TEMPORAL": "2", "MP_RANDOM": "1", "MP_X_HALO_ALIGN": "1"})
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "jacobi bad 0" in out


def test_exchange_random_radius_maps_device(st):
    """property test on the device: random radius maps, sizes, 1-4 sub-domains per GPU, element
    types and x layouts, through a random same-process transport (direct stores, DMA-engine pipes, host-staged)"""
    from hypothesis import HealthCheck, given, settings
    from hypothesis import strategies as hs
    from test_exchange_property import exchange_case, _radius

    @settings(max_examples=15, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
    @given(exchange_case(), hs.sampled_from(["Kernel", "PeerCopy", "PeerCopyEngine", "Staged"]))
    def run(case, method):
        radii, n, size, dtype, align = case
        radius = _radius(st, radii)
        tr = st.TransportOptions()
        if method == "PeerCopyEngine":
            tr.peer_copy = st.TransportOptions.Copy.Engine
            method = "PeerCopy"
        dd = st.DistributedDomain(*size, group=st.make_single_group())
        dd.set_transport_options(tr)
        dd.set_radius(radius)
        dd.set_gpus([0] * n)
        dd.set_methods(getattr(st.MethodFlags, method))
        dd.set_x_halo_align(align)
        q = dd.add_data("q", dtype)
        dd.realize()
        for it in range(2):
            fill_coords(dd, q, offset=it)
            dd.exchange()
            assert check_exchange(dd, q, radius, offset=it) == 0, (case, method)
            dd.swap()

    run()


@pytest.mark.parametrize("kind,size,gpus,temporal", [("jacobi", (512, 120, 116), [0], 2), ("jacobi", (64, 36, 30), [0, 0], 2),
                                                     ("astaroth", (512, 16, 24), [0], 2), ("jacobi", (48, 40, 36), [0, 0, 0], 1)])
def test_interior_align_128_models(st, kind, size, gpus, temporal):
    """interior_align=128: every row's first interior cell on an L2-line boundary; kernels unchanged, bitwise"""
    from stencil2_amd.ops import astaroth_step_reference
    cls, ref, kw = ((st.Jacobi3D, jacobi_step_reference, {}) if kind == "jacobi"
                    else (st.AstarothSim, astaroth_step_reference, {"quantities": 2}))
    m = cls(size, gpus=gpus, temporal=temporal, interior_align=128, **kw)
    m.init()
    d = m.domain.domain(0)
    assert (d.curr_ptr(0) + d.radius().x(-1) * d.elem_size(0)) % 128 == 0
    assert m.temporal_blocking() == (temporal == 2)
    u = _gather(m)
    m.run(5)
    for _ in range(5):
        u = ref(u)
    m.synchronize()
    assert torch.equal(_gather(m), u)


@pytest.mark.parametrize("rname", ["r1", "r3", "fec", "asym"])
@pytest.mark.parametrize("gpus,size", [([0], (64, 13, 11)), ([0, 0], (128, 13, 11)), ([0, 0, 0], (32, 13, 11))])
def test_x_face_lines_device(st, rname, gpus, size):
    """TransportOptions.x_face_sectors on the device: same-GPU x faces as whole 128-B lines, exact halos"""
    radius = _radii(st)[rname]
    tr = st.TransportOptions()
    tr.x_face_sectors = True
    for dtype in (torch.float32, torch.float64):
        dd, q = _dd(st, size, radius, gpus, st.MethodFlags.Kernel, dtype=dtype, transport=tr)
        for it in range(2):
            fill_coords(dd, q, offset=it)
            dd.exchange()
            assert check_exchange(dd, q, radius, offset=it) == 0
            dd.swap()


@pytest.mark.parametrize("rname", ["r1", "r3", "fec"])
@pytest.mark.parametrize("gpus,size", [([0], (64, 13, 11)), ([0, 0], (128, 13, 11))])
def test_x_face_lines_auto_device(st, rname, gpus, size):
    """TransportOptions.x_face_lines_auto_bytes: a GPU's same-GPU x faces switch to whole lines once their lines
    reach the threshold (1 B here, so always; prepare_skip_wrapped's subset too), exact halos"""
    radius = _radii(st)[rname]
    tr = st.TransportOptions()
    tr.x_face_lines_auto_bytes = 1
    for dtype in (torch.float32, torch.float64):
        dd, q = _dd(st, size, radius, gpus, st.MethodFlags.Kernel, dtype=dtype, transport=tr)
        for it in range(2):
            fill_coords(dd, q, offset=it)
            dd.exchange()
            assert check_exchange(dd, q, radius, offset=it) == 0
            dd.swap()


@pytest.mark.parametrize("kind,fp64", [("jacobi", False), ("astaroth", False), ("jacobi", True)])
def test_ops_stencil7x2_apply_on_a_domain(st, kind, fp64):
    """ops.stencil7x2_apply on a user's DistributedDomain: exchange the depth-2 halos, one fused call = two steps of
    the torch oracle, bitwise; the same with the periodic image read in-kernel (tune.wrap = 7, no exchange)"""
    from stencil2_amd.ops import astaroth_step_reference, stencil7x2_apply, stencil7x2_supported
    K = st.StencilKind.Jacobi if kind == "jacobi" else st.StencilKind.Astaroth
    ref = jacobi_step_reference if kind == "jacobi" else astaroth_step_reference
    dtype = torch.float64 if fp64 else torch.float32
    L = (64, 48, 40)
    for wrap in (0, 7):
        dd = st.DistributedDomain(*L, group=st.make_single_group())
        dd.set_radius(st.Radius.face_edge_corner(2, 1, 0))
        dd.set_gpus([0])
        q = dd.add_data("u", dtype)
        dd.realize()
        assert stencil7x2_supported(dd, 0, q)
        u = torch.rand((L[2], L[1], L[0]), generator=torch.Generator().manual_seed(5), dtype=torch.float64).to(dtype)
        dd.curr_interior(0, q).copy_(u.cuda())
        torch.cuda.synchronize()
        if wrap == 0:
            dd.exchange()
        t = st.StencilTune()
        t.wrap = wrap
        stencil7x2_apply(dd, 0, q, dd.domain(0).get_compute_region(), K, spheres=kind == "jacobi", tune=t)
        torch.cuda.synchronize()
        dd.swap()
        want = ref(ref(u.cuda()))
        assert torch.equal(dd.curr_interior(0, q), want), f"wrap {wrap}"
