"""Halo exchange on the CPU backend (BASELINE config #1 path: no GPU, 1 rank) with the analytic coordinate oracle.
Covers the reference's test_exchange.cu radius patterns plus its coverage gaps: asymmetric radii on the
same-device path, edge/corner-only radii, uneven partitions, mixed element sizes, several sub-domains per process."""
import pytest
import torch

from stencil2_amd.utils.testing import check_exchange, fill_coords


def radius_patterns(st):
    pats = {}
    pats["r0"] = st.Radius.constant(0)
    pats["r1"] = st.Radius.constant(1)
    pats["r2"] = st.Radius.constant(2)
    r = st.Radius.constant(0); r.set_dir(1, 0, 0, 2); pats["+x2"] = r
    r = st.Radius.constant(0); r.set_dir(-1, 0, 0, 1); pats["-x1"] = r
    r = st.Radius.constant(0); r.set_dir(1, 0, 0, 2); r.set_dir(-1, 0, 0, 1); pats["+x2-x1"] = r
    r = st.Radius.constant(0); r.set_face(1); pats["faces"] = r
    pats["fec"] = st.Radius.face_edge_corner(2, 1, 0)
    pats["corners"] = st.Radius.face_edge_corner(1, 0, 1)
    r = st.Radius.constant(0); r.set_face(2); r.set_dir(1, 1, 0, 2); pats["faces+1edge"] = r
    r = st.Radius.constant(1); r.set_dir(0, 0, 1, 3); r.set_dir(0, -1, 0, 2); pats["mixed"] = r
    return pats


def make_dd(st, size, radius, gpus, methods=None, dtype=torch.int64, nq=1, backend=None, transport=None):
    dd = st.DistributedDomain(*size, group=st.make_single_group())
    dd.set_backend(backend or st.Backend.Host)
    if transport is not None:
        dd.set_transport_options(transport)
    dd.set_radius(radius)
    dd.set_gpus(gpus)
    if methods is not None:
        dd.set_methods(methods)
    qs = [dd.add_data(f"q{i}", dtype) for i in range(nq)]
    dd.realize()
    return dd, qs


@pytest.mark.parametrize("name", ["r0", "r1", "r2", "+x2", "-x1", "+x2-x1", "faces", "fec", "corners",
                                  "faces+1edge", "mixed"])
@pytest.mark.parametrize("gpus", [[0], [0, 0], [0, 0, 0]])
def test_exchange_patterns(st, name, gpus):
    radius = radius_patterns(st)[name]
    dd, (q,) = make_dd(st, (13, 11, 9), radius, gpus)
    fill_coords(dd, q)
    dd.exchange()
    assert check_exchange(dd, q, radius) == 0


@pytest.mark.parametrize("gpus", [[0, 0], [0, 0, 0, 0]])
def test_exchange_staged_only_same_process(st, gpus):
    """Staged transport between sub-domains of one process (loopback through the process group)."""
    radius = st.Radius.constant(1)
    dd, (q,) = make_dd(st, (12, 10, 8), radius, gpus, methods=st.MethodFlags.Staged)
    fill_coords(dd, q)
    dd.exchange()
    assert check_exchange(dd, q, radius) == 0
    assert dd.exchange_bytes_for_method(st.MethodFlags.Staged) > 0


def test_exchange_mixed_dtypes_multi_quantity(st):
    radius = st.Radius.constant(2)
    dd = st.DistributedDomain(10, 9, 8, group=st.make_single_group())
    dd.set_backend(st.Backend.Host)
    dd.set_radius(radius)
    dd.set_gpus([0, 0])
    qa = dd.add_data("a", torch.int64)
    qb = dd.add_data("b", torch.int32)
    qc = dd.add_data("c", torch.float64)
    dd.realize()
    for q in (qa, qb, qc):
        fill_coords(dd, q)
    dd.exchange()
    for q in (qa, qb, qc):
        assert check_exchange(dd, q, radius) == 0


def test_exchange_swap_parity(st):
    """Exchanges act on the current buffer after any number of swaps."""
    radius = st.Radius.constant(1)
    dd, (q,) = make_dd(st, (8, 8, 8), radius, [0, 0])
    for it in range(3):
        fill_coords(dd, q)
        dd.exchange()
        assert check_exchange(dd, q, radius) == 0
        dd.swap()


def test_exchange_interior_untouched_and_bytes(st):
    radius = st.Radius.constant(1)
    dd, (q,) = make_dd(st, (64, 64, 64), radius, [0], dtype=torch.float32)
    dd.fill_from_global(q, lambda z, y, x: (x + 3 * y + 7 * z).float())
    before = dd.curr_interior(0, q).clone()
    dd.exchange()
    assert torch.equal(before, dd.curr_interior(0, q))
    # BASELINE config #1: 64^3 radius-1, 26 directions: 101408 B per quantity
    assert dd.exchange_bytes_for_method(st.MethodFlags.All) == 101408


def test_interior_exterior_partition(st):
    """get_interior/get_exterior tile the compute region without overlap (reference stencil.cu:567-666)."""
    for radius in (st.Radius.constant(1), radius_patterns(st)["+x2-x1"], radius_patterns(st)["mixed"]):
        dd, (q,) = make_dd(st, (12, 10, 9), radius, [0, 0])
        ins, exts = dd.get_interior(), dd.get_exterior()
        for di in range(dd.num_domains()):
            cr = dd.domain(di).get_compute_region()
            cover = torch.zeros(cr.extent().z, cr.extent().y, cr.extent().x, dtype=torch.int32)
            for reg in [ins[di], *exts[di]]:
                lo, hi = reg.lo - cr.lo, reg.hi - cr.lo
                if hi.x > lo.x and hi.y > lo.y and hi.z > lo.z:
                    cover[lo.z:hi.z, lo.y:hi.y, lo.x:hi.x] += 1
            assert int(cover.min()) == 1 and int(cover.max()) == 1


def test_plan_summary_and_methods(st):
    radius = st.Radius.constant(1)
    dd, _ = make_dd(st, (16, 8, 8), radius, [0, 0])
    s = dd.plan_summary()
    assert "== kernel ==" in s
    assert all(e.method == st.MethodFlags.Kernel for e in dd.plan())
    assert len(dd.plan()) == 2 * 26
    assert st.methods_to_string(st.MethodFlags.All) == "staged/rccl/colo/peer/kernel"


@pytest.mark.parametrize("axes", [(False, True, True), (True, False, True), (False, False, False), (True, True, False)])
@pytest.mark.parametrize("gpus", [[0], [0, 0, 0, 0]])
def test_exchange_nonperiodic(st, axes, gpus):
    """Boundary (reference include/stencil/boundary.hpp, unused there): no halo crosses a non-periodic face."""
    radius = st.Radius.face_edge_corner(2, 1, 1)
    b = st.Boundary.axes(*axes)
    dd = st.DistributedDomain(13, 11, 9, group=st.make_single_group())
    dd.set_backend(st.Backend.Host)
    dd.set_radius(radius)
    dd.set_boundary(b)
    dd.set_gpus(gpus)
    q = dd.add_data("q", torch.int64)
    dd.realize()
    fill_coords(dd, q)
    dd.exchange()
    assert check_exchange(dd, q, radius, boundary=b) == 0


def test_native_ctest_cpu():
    """The native C++ unit tests (stencil_ctest, CPU cases: geometry, partition, QAP, tags, Array, host exchange)."""
    import os
    import subprocess
    exe = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "bin", "stencil_ctest")
    if not os.path.exists(exe):
        pytest.skip("native tests not built")
    r = subprocess.run([exe, "--cpu"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("gpus", [[0], [0, 0], [0, 0, 0, 0]])
@pytest.mark.parametrize("axes", [(True, True, True), (False, True, True), (True, True, False)])
def test_self_wrap_axes(st, gpus, axes):
    """self_wrap_axes: exactly the periodic axes the decomposition leaves whole (each sub-domain its own neighbour
    there) -- the axes StencilModel's fused pairs read periodically in-kernel instead of copying halos."""
    dd = st.DistributedDomain(24, 20, 16, group=st.make_single_group())
    dd.set_backend(st.Backend.Host)
    dd.set_radius(2)
    dd.set_boundary(st.Boundary.axes(*axes))
    dd.set_gpus(gpus)
    q = dd.add_data("q", torch.int64)
    dd.realize()
    pd = dd.placement_dim()
    want = sum(1 << a for a, (n, p) in enumerate(zip((pd.x, pd.y, pd.z), axes)) if n == 1 and p)
    assert dd.self_wrap_axes() == want
    dd.prepare_skip_wrapped(want)  # host backend: the full exchange runs (nothing to skip on the host path)
    fill_coords(dd, q)
    dd.exchange_async(0, want)
    r = st.Radius.constant(2)
    assert check_exchange(dd, q, r, boundary=st.Boundary.axes(*axes)) == 0
    if want != 7:
        with pytest.raises(Exception):
            dd.prepare_skip_wrapped(7 & ~want)


def test_select_method_priority_and_shared_gpu(st):
    """Transport ladder (reference src/stencil.cu:163-194) as a pure function, including the pair-scoped RCCL
    fallback: only pairs with an endpoint on a GPU that two ranks drive leave RCCL (for the staged path)."""
    M = st.MethodFlags
    sel = st._C.select_method
    assert sel(M.All, same_rank=True, same_device=True) == M.Kernel
    assert sel(M.All, same_rank=True, peer=True) == M.PeerCopy
    assert sel(M.All, same_host=True, can_access=True) == M.Colocated
    assert sel(M.All, same_host=True, can_access=False) == M.Rccl
    assert sel(M.All) == M.Rccl  # other host
    # shared GPU: Colocated still wins when IPC works; otherwise staged, never RCCL
    assert sel(M.All, same_host=True, can_access=True, shared_gpu=True) == M.Colocated
    assert sel(M.All, same_host=True, shared_gpu=True) == M.Staged
    assert sel(M.Rccl | M.Kernel, same_host=True, shared_gpu=True) == M.Staged
    # a pair between two exclusive GPUs of the same job keeps RCCL
    assert sel(M.Rccl | M.Kernel, same_host=True, shared_gpu=False) == M.Rccl
    assert sel(M.Kernel) == M.None_
    # host backend: translate within a process, staged across processes
    assert sel(M.All, device=False, same_rank=True, same_device=True) == M.Kernel
    assert sel(M.All, device=False) == M.Staged
    assert sel(M.Kernel, device=False) == M.None_


def test_x_face_lines_auto_default(st):
    """whole-line x faces switch on by themselves from 128 MiB of x-face lines per GPU (measured crossover between
    96 and 192 MiB, below the 256-MB last-level cache)"""
    tr = st.TransportOptions()
    assert tr.x_face_lines_auto_bytes == 128 << 20 and not tr.x_face_sectors


@pytest.mark.parametrize("name", ["r1", "r2", "+x2", "-x1", "+x2-x1", "fec", "mixed"])
@pytest.mark.parametrize("size,gpus", [((64, 12, 10), [0]), ((64, 12, 10), [0, 0]), ((32, 10, 9), [0, 0, 0]),
                                       ((30, 10, 9), [0])])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_exchange_x_face_sectors(st, name, size, gpus, dtype):
    """TransportOptions.x_face_sectors: same-process x faces copied as whole 128-B lines (the interior-alignment unit;
    the extra cells go to the receiver's row padding) give exactly the same halos; x extents that are no multiple of
    a line fall back."""
    radius = radius_patterns(st)[name]
    tr = st.TransportOptions()
    tr.x_face_sectors = True
    dd, (q,) = make_dd(st, size, radius, gpus, dtype=dtype, transport=tr)
    for it in range(2):
        fill_coords(dd, q, offset=it)
        dd.exchange()
        assert check_exchange(dd, q, radius, offset=it) == 0
        dd.swap()


@pytest.mark.parametrize("name", ["r1", "r2", "+x2-x1", "fec", "mixed"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.int64])
@pytest.mark.parametrize("gpus", [[0], [0, 0, 0]])
def test_exchange_x_halo_aligned_layout(st, name, dtype, gpus):
    """Halo-aligned x layout (LocalDomain.set_x_halo_align): the interior starts 16-B aligned inside
    its row's first 64-B sector with the -x halo directly in front, rows stay 128-B aligned; the exchange is exact."""
    radius = radius_patterns(st)[name]
    dd = st.DistributedDomain(13, 11, 9, group=st.make_single_group())
    dd.set_backend(st.Backend.Host)
    dd.set_radius(radius)
    dd.set_gpus(gpus)
    dd.set_x_halo_align(True)
    q = dd.add_data("q", dtype)
    dd.realize()
    for di in range(dd.num_domains()):
        d = dd.domain(di)
        es = d.elem_size(q)
        rx = d.radius().x(-1)
        raw0 = d.curr_ptr(q)
        first = raw0 + rx * es  # first interior cell
        assert first % 16 == 0 and (first // 64) == ((raw0 - 0) // 64 if rx * es <= 16 else (first - 1) // 64)
        assert (raw0 - d.pad_x(q) * es) % 128 == 0 and (d.pitch(q).x * es) % 128 == 0
        assert d.front_slack(q) == d.pad_x(q) + 128 // es
        assert d.x_halo_align()
    fill_coords(dd, q)
    dd.exchange()
    assert check_exchange(dd, q, radius) == 0


@pytest.mark.parametrize("name", ["r1", "r2", "+x2", "-x1", "+x2-x1", "fec", "mixed"])
@pytest.mark.parametrize("gpus", [[0], [0, 0]])
@pytest.mark.parametrize("dtype", [torch.int64, torch.float32])
def test_exchange_shared_halo_lines(st, name, gpus, dtype):
    """Shared halo lines (LocalDomain.set_shared_halo_line): the row pitch is the raw row rounded
    up to whole 128-B lines, so row r's +x halo and row r+1's -x halo share a line and a row's raw cells reach into
    the next row's front padding. Every halo still lands on its own cell (coordinate oracle, 3 exchanges with swaps),
    the interiors stay line-aligned, and the pitch is one line shorter than the default layout's."""
    radius = radius_patterns(st)[name]
    size = (64, 11, 9)
    dd = st.DistributedDomain(*size, group=st.make_single_group())
    dd.set_backend(st.Backend.Host)
    dd.set_radius(radius)
    dd.set_gpus(gpus)
    dd.set_shared_halo_line(True)
    q = dd.add_data("q", dtype)
    dd.realize()
    ref, _ = make_dd(st, size, radius, gpus, dtype=dtype)
    for di in range(dd.num_domains()):
        d, r = dd.domain(di), ref.domain(di)
        assert d.shared_halo_line()
        es = torch.empty((), dtype=dtype).element_size()
        assert d.pitch(0).x * es % 128 == 0 and (d.pad_x(0) + d.radius().x(-1)) * es % 128 == 0
        assert d.raw_size().x <= d.pitch(0).x < d.raw_size().x + 128 // es
        assert d.pitch(0).x <= r.pitch(0).x - (128 // es if d.radius().x(-1) and d.radius().x(1) else 0)
        assert d.row_limit(0) == d.pitch(0).x
    for it in range(3):
        fill_coords(dd, q, offset=it)
        dd.exchange()
        assert check_exchange(dd, q, radius, offset=it) == 0
        dd.swap()


def test_shared_halo_line_translate_pairs_one_line(st):
    """Depth-2 face self-exchange on a shared-halo-line domain: the x-face translates are split into the rows that
    pair up line by line (row y's +x halo with row y+1's -x halo) and the one row per plane that has no partner in
    its face; every halo cell still arrives."""
    dd = st.DistributedDomain(64, 8, 4, group=st.make_single_group())
    dd.set_backend(st.Backend.Host)
    r = st.Radius.constant(0)
    r.set_face(2)
    dd.set_radius(r)
    dd.set_shared_halo_line(True)
    q = dd.add_data("q", torch.float32)
    dd.realize()
    fill_coords(dd, q)
    dd.exchange()
    assert check_exchange(dd, q, r) == 0
