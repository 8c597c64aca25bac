"""Geometry primitives. Expectations from reference test/test_cpu_radius.cpp, test_cuda_local_domain.cu,
test_cuda_packer.cu (264-byte layout) and the fixed Dim3 bugs."""
import pytest


def test_radius_constant_and_faces(st):
    r = st.Radius.constant(3)
    assert r.dir(1, -1, 1) == 3 and r.x(-1) == 3
    r2 = st.Radius.constant(0)
    r2.set_face(2)
    assert r2.x(1) == 2 and r2.y(-1) == 2 and r2.z(1) == 2 and r2.dir(1, 1, 0) == 0
    fec = st.Radius.face_edge_corner(3, 2, 1)
    assert fec.dir(0, 0, 0) == 0 and fec.dir(1, 0, 0) == 3 and fec.dir(0, 1, 1) == 2 and fec.dir(-1, -1, 1) == 1
    assert fec.max() == 3


def test_dim3_fixed_reference_bugs(st):
    assert st.Dim3(1, 5, 3).max() == 5  # reference max() compared x only
    assert st.Dim3(1, 2, 3) != st.Dim3(1, 2, 4)  # reference operator!= tested z == rhs.z
    assert st.Dim3(-1, 5, 10).wrap(st.Dim3(4, 4, 4)) == st.Dim3(3, 1, 2)
    assert st.Dim3(1, 2, 3).flatten() == 6


def _ld(st, sz, r, dtypes=((4, "F32"),)):
    from stencil2_amd import _C

    ld = _C.LocalDomain(st.Dim3(*sz), st.Dim3(0, 0, 0), -1, st.Backend.Host)
    ld.set_radius(r)
    for es, dt in dtypes:
        ld.add_data(es, "", getattr(st.DType, dt))
    ld.realize()
    return ld


def test_local_domain_symmetric_radius_positions(st):
    ld = _ld(st, (30, 40, 50), st.Radius.constant(4), ((8, "F64"),))
    D = st.Dim3
    # faces in halo / compute (reference test_cuda_local_domain.cu:34-52)
    assert ld.halo_pos(D(-1, 0, 0), True) == D(0, 4, 4)
    assert ld.halo_pos(D(1, 0, 0), True) == D(34, 4, 4)
    assert ld.halo_pos(D(0, 1, 0), True) == D(4, 44, 4)
    assert ld.halo_pos(D(0, 0, 1), True) == D(4, 4, 54)
    assert ld.halo_pos(D(1, 0, 0), False) == D(30, 4, 4)
    assert ld.halo_pos(D(0, 0, 1), False) == D(4, 4, 50)
    assert ld.halo_pos(D(-1, 0, 0), False) == D(4, 4, 4)
    # extents
    assert ld.halo_extent(D(-1, 0, 0)) == D(4, 40, 50)
    assert ld.halo_extent(D(0, -1, 0)) == D(30, 4, 50)
    assert ld.halo_extent(D(1, 1, 0)) == D(4, 4, 50)
    assert ld.halo_extent(D(1, 1, 1)) == D(4, 4, 4)
    # edges / corners
    assert ld.halo_pos(D(1, -1, 0), True) == D(34, 0, 4)
    assert ld.halo_pos(D(0, 1, 1), True) == D(4, 44, 54)
    assert ld.halo_pos(D(1, 1, 1), True) == D(34, 44, 54)
    assert ld.halo_pos(D(1, 1, 1), False) == D(30, 40, 50)
    assert ld.raw_size() == D(38, 48, 58)


def test_local_domain_x_leaning_radius(st):
    r = st.Radius.constant(0)
    r.set_dir(1, 0, 0, 3)
    ld = _ld(st, (30, 40, 50), r, ((4, "I32"),))
    D = st.Dim3
    assert ld.halo_pos(D(-1, 0, 0), True) == D(0, 0, 0)
    assert ld.halo_pos(D(1, 0, 0), True) == D(30, 0, 0)
    assert ld.halo_extent(D(1, 0, 0)) == D(3, 40, 50)
    assert ld.halo_extent(D(-1, 0, 0)) == D(0, 40, 50)
    assert ld.halo_extent(D(0, 1, 0)) == D(30, 0, 50)


def test_packed_layout_264_bytes(st):
    """reference test_cuda_packer.cu:69-91: float+char+double, +x radius 2 / -x radius 1, send +x -> 264 B"""
    from stencil2_amd import _C

    r = st.Radius.constant(0)
    r.set_dir(1, 0, 0, 2)
    r.set_dir(-1, 0, 0, 1)
    ld = _ld(st, (3, 4, 5), r, ((4, "F32"), (1, "I8"), (8, "F64")))
    assert _C.packed_message_bytes(ld, [st.Dim3(1, 0, 0)]) == 264
    # both directions: 20*(4+1+8) aligned + 40*(4+1+8)... order-independent of the input list
    a = _C.packed_message_bytes(ld, [st.Dim3(-1, 0, 0), st.Dim3(1, 0, 0)])
    b = _C.packed_message_bytes(ld, [st.Dim3(1, 0, 0), st.Dim3(-1, 0, 0)])
    assert a == b and a > 264


def test_padded_pitch_alignment(st):
    """x pitch padded so the first interior x of every row is 128-B aligned (one L2 line), or 64-B
    with set_interior_align(64)."""
    for rx in (1, 2, 3, 5):
        ld = _ld(st, (37, 5, 4), st.Radius.constant(rx), ((4, "F32"), (8, "F64")))
        for q, es in ((0, 4), (1, 8)):
            p = ld.pitch(q)
            assert (p.x * es) % 128 == 0
            assert ((ld.pad_x(q) + rx) * es) % 128 == 0
            assert p.x >= ld.pad_x(q) + ld.raw_size().x + 16 // es + 1


def test_x2_lockstep_schedule(st):
    """whole-row fused-pair block schedule: quarters over 64 row groups of 512^3, quarters plus second segments when
    more row groups than slots / 4 (the overlap's 248 slots, 645x645x323), P = slots / groups parts over every row
    group when fewer (813x407x407, 645x323x645)"""
    f = st._C.x2_lockstep_schedule
    assert f(256, 64, 512) == (4, 256, 1)     # 512^3: 64 row groups of 8, quarters
    assert f(248, 64, 508) == (4, 248, 1)     # overlap interior: 62 groups in lockstep, 2 as second segments
    assert f(256, 51, 407) == (5, 255, 1)     # 813x407x407: 51 groups x 5 parts of 81-82 planes
    assert f(256, 81, 323) == (4, 256, 1)     # 645x645x323 (odd): quarters over 64 groups + 17 as second segments
    assert f(256, 102, 204) == (5, 255, 2)    # 813x813x204: 2 rounds x 51 groups x 5 parts
    assert f(256, 70, 512) == (7, 245, 2)     # 2 rounds x 35 groups x 7 parts (245 >= 15/16 of 256)
    assert f(256, 41, 645) == (6, 246, 1)     # 645x323x645
    assert f(256, 128, 256) == (2, 256, 1)    # 1024x512x256 (512-cell columns: 2 x 64): two parts over whole columns
    assert f(256, 256, 256) == (1, 256, 1)    # one block per column
    assert f(256, 300, 512) == (1, 150, 2)    # more columns than slots: 2 rounds of whole columns on 150 blocks
    assert f(256, 512, 1024) == (1, 256, 2)   # fp64 1024^3: 4 x 128 columns, 2 rounds
    assert f(256, 64, 40) == (0, 0, 1)        # thin grids: balanced split
    assert f(256, 17, 200) == (0, 0, 1)       # 15 parts of 13 planes: too short


def test_interior_align_64_option(st):
    """set_interior_align(64): the rounds-1-3 layout, first interior x on a 64-B sector"""
    from stencil2_amd import _C
    for rx in (1, 2, 3):
        ld = _C.LocalDomain(st.Dim3(37, 5, 4), st.Dim3(0, 0, 0), -1, st.Backend.Host)
        ld.set_radius(st.Radius.constant(rx))
        ld.set_interior_align(64)
        ld.add_data(4, "", st.DType.F32)
        ld.realize()
        assert ld.interior_align() == 64
        assert ((ld.pad_x(0) + rx) * 4) % 64 == 0 and ld.pad_x(0) < 16 and (ld.pitch(0).x * 4) % 128 == 0
