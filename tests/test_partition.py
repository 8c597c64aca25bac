"""Partitioning and QAP placement. Expected values from reference test/test_cpu_partition.cpp and
test/test_cpu_qap.cpp; NodeAware with fake topologies (the reference has no test for it)."""
import math
import random

import pytest
from hypothesis import given, settings, strategies as hs


def test_rank_partition_reference_values(st):
    D = st.Dim3
    p = st.RankPartition(D(10, 5, 5), 2)
    assert p.dim() == D(2, 1, 1)
    assert p.subdomain_size(D(0, 0, 0)) == D(5, 5, 5) and p.subdomain_size(D(1, 0, 0)) == D(5, 5, 5)
    p = st.RankPartition(D(10, 3, 1), 4)
    assert [p.subdomain_size(D(i, 0, 0)) for i in range(4)] == [D(3, 3, 1), D(3, 3, 1), D(2, 3, 1), D(2, 3, 1)]
    assert [p.subdomain_origin(D(i, 0, 0)) for i in range(4)] == [D(0, 0, 0), D(3, 0, 0), D(6, 0, 0), D(8, 0, 0)]
    p = st.RankPartition(D(10, 5, 5), 3)
    assert [p.subdomain_size(D(i, 0, 0)) for i in range(3)] == [D(4, 5, 5), D(3, 5, 5), D(3, 5, 5)]
    p = st.RankPartition(D(13, 7, 7), 4)
    assert [p.subdomain_size(D(i, 0, 0)) for i in range(4)] == [D(4, 7, 7), D(3, 7, 7), D(3, 7, 7), D(3, 7, 7)]
    p = st.RankPartition(D(10, 14, 2), 9)
    assert p.subdomain_origin(D(0, 0, 0)) == D(0, 0, 0)
    assert p.subdomain_origin(D(1, 1, 0)) == D(4, 5, 0)
    assert p.subdomain_origin(D(2, 2, 0)) == D(7, 10, 0)


def test_node_partition_min_interface(st):
    D = st.Dim3
    r = st.Radius.constant(0)
    r.set_face(1)
    p = st.NodePartition(D(1024, 1024, 1024), r, 1, 8)
    assert p.dim() == D(2, 2, 2)
    assert p.subdomain_size(D(1, 1, 1)) == D(512, 512, 512)
    # weak-scaling sizes of the reference: 645 -> 323 + 322; ties cut z first (contiguous faces)
    p = st.NodePartition(D(645, 645, 645), r, 1, 2)
    assert p.dim() == D(1, 1, 2)
    assert p.subdomain_size(D(0, 0, 0)) == D(645, 645, 323) and p.subdomain_size(D(0, 0, 1)) == D(645, 645, 322)
    p = st.NodePartition(D(813, 813, 813), r, 1, 4)
    assert p.dim() == D(1, 2, 2)
    # x-only radius: cuts avoid the x interface (x-interface weight large)
    rx = st.Radius.constant(0)
    rx.set_dir(1, 0, 0, 4)
    rx.set_dir(-1, 0, 0, 4)
    p = st.NodePartition(D(100, 100, 100), rx, 2, 2)
    assert p.dim().x == 1
    # the models' MI355X cut costs (x faces count double): weak-scaled cubes are never cut along x up to 8 GPUs,
    # with the same face bytes per GPU (1x2x4 of 1024^3: 3 links x 4 MiB, like 2x2x2)
    c = D(2, 1, 1)
    assert st.NodePartition(D(1024, 1024, 1024), r, 1, 8, c).dim() == D(1, 2, 4)
    assert st.NodePartition(D(813, 813, 813), r, 1, 4, c).dim() == D(1, 2, 2)
    assert st.NodePartition(D(645, 645, 645), r, 1, 2, c).dim() == D(1, 1, 2)
    # the models' default (4, 3, 2): equal face area, z cuts preferred (contiguous faces; the whole-row sweeps are
    # faster with long y: 1024x512x256 1000 vs 1024x256x512 972, 645x645x323 837 vs 645x323x645 790 Gcells/s)
    c = D(4, 3, 2)
    assert st.NodePartition(D(1024, 1024, 1024), r, 1, 8, c).dim() == D(1, 2, 4)
    assert st.NodePartition(D(813, 813, 813), r, 1, 4, c).dim() == D(1, 2, 2)
    assert st.NodePartition(D(645, 645, 645), r, 1, 2, c).dim() == D(1, 1, 2)
    # the round-1 default (4, 2, 3): y cuts preferred
    c = D(4, 2, 3)
    assert st.NodePartition(D(1024, 1024, 1024), r, 1, 8, c).dim() == D(1, 4, 2)
    assert st.NodePartition(D(813, 813, 813), r, 1, 4, c).dim() == D(1, 2, 2)
    assert st.NodePartition(D(645, 645, 645), r, 1, 2, c).dim() == D(1, 2, 1)
    assert st.NodePartition(D(1024, 1024, 1024), r, 1, 8, D(1, 1, 1)).dim() == D(2, 2, 2)


@settings(max_examples=60, deadline=None)
@given(hs.integers(1, 40), hs.integers(1, 40), hs.integers(1, 40), hs.integers(1, 12))
def test_rank_partition_tiles_domain(st, x, y, z, n):
    D = st.Dim3
    p = st.RankPartition(D(x, y, z), n)
    dim = p.dim()
    if dim.x > x or dim.y > y or dim.z > z:
        return  # more parts than cells in an axis: not a valid decomposition request
    covered = 0
    for k in range(dim.flatten()):
        idx = p.dimensionize(k)
        s, o = p.subdomain_size(idx), p.subdomain_origin(idx)
        assert s.x > 0 and s.y > 0 and s.z > 0
        covered += s.flatten()
        # contiguous tiling along each axis
        if idx.x + 1 < dim.x:
            assert p.subdomain_origin(D(idx.x + 1, idx.y, idx.z)).x == o.x + s.x
    assert covered == x * y * z


INF = math.inf


def test_qap_reference_triangle(st):
    bw = [[INF, 1, 10], [1, INF, 1], [10, 1, INF]]
    comm = [[0, 10, 1], [10, 0, 1], [1, 1, 0]]
    f, _ = st.qap_solve(comm, st.make_reciprocal(bw))
    assert list(f) == [0, 2, 1]


P9_BW = [[900, 75, 64, 64], [75, 900, 64, 64], [64, 64, 900, 75], [64, 64, 75, 900]]
P9_COMM = [[7, 5, 10, 1], [5, 7, 1, 10], [10, 1, 7, 5], [1, 10, 5, 7]]


def test_qap_reference_p9(st):
    f, _ = st.qap_solve(P9_COMM, st.make_reciprocal(P9_BW))
    assert list(f) == [0, 2, 1, 3]


def test_qap_reference_p9_catch(st):
    f, _ = st.qap_solve_catch(P9_COMM, st.make_reciprocal(P9_BW))
    assert list(f) == [3, 1, 2, 0]


def test_qap_big_catch_smoke_and_optimality(st):
    rng = random.Random(0)
    n = 64
    bw = [[rng.random() * 100 + 1 for _ in range(n)] for _ in range(n)]
    comm = [[rng.random() for _ in range(n)] for _ in range(n)]
    f, c = st.qap_solve_catch(comm, st.make_reciprocal(bw))
    assert sorted(f) == list(range(n))
    assert c <= st.qap_cost(comm, st.make_reciprocal(bw), list(range(n))) + 1e-9
    # small instances: local search never beats exhaustive
    for trial in range(5):
        m = 6
        bw = [[rng.random() * 10 + 1 for _ in range(m)] for _ in range(m)]
        comm = [[rng.random() for _ in range(m)] for _ in range(m)]
        d = st.make_reciprocal(bw)
        fe, ce = st.qap_solve(comm, d)
        fc, cc = st.qap_solve_catch(comm, d)
        assert ce <= cc + 1e-12
        assert abs(st.qap_cost(comm, d, list(fe)) - ce) < 1e-9


def test_trivial_and_nodeaware_single_process(st):
    g = st.make_single_group()
    D = st.Dim3
    r = st.Radius.constant(1)
    t = st.TrivialPlacement(D(20, 10, 10), g, [0, 1, 2, 3])
    assert t.dim() == D(4, 1, 1)
    assert [t.get_device(t.get_idx(0, i)) for i in range(4)] == [0, 1, 2, 3]
    # uniform mesh: QAP is degenerate -> deterministic identity mapping
    na = st.NodeAwarePlacement(D(64, 64, 64), g, r, list(range(8)), lambda a, b: 10.0 if a == b else 1.0)
    assert na.dim() == D(2, 2, 2)
    assert [na.get_subdomain_id(na.get_idx(0, i)) for i in range(8)] == list(range(8))
    # a topology with two tight pairs: heavy-traffic neighbours land on the close pair
    def bw(a, b):
        if a == b:
            return 100.0
        return 50.0 if a // 2 == b // 2 else 1.0
    rx = st.Radius.constant(0)
    rx.set_dir(1, 0, 0, 8)
    rx.set_dir(-1, 0, 0, 8)
    rx.set_dir(0, 1, 0, 1)
    rx.set_dir(0, -1, 0, 1)
    na = st.NodeAwarePlacement(D(64, 64, 8), g, rx, [0, 1, 2, 3], bw)
    dim = na.dim()
    assert dim.flatten() == 4
    # every pair of x-neighbours (heaviest traffic) shares a tight pair
    for k in range(4):
        idx = st.Dim3(k % dim.x, (k // dim.x) % dim.y, 0)
        nb = st.Dim3((idx.x + 1) % dim.x, idx.y, 0)
        if dim.x > 1:
            assert na.get_device(idx) // 2 == na.get_device(nb) // 2


def test_node_partition_max_link(st):
    """PartitionObjective.MaxLink: the node's GPUs are a fully connected xGMI mesh, so the cut minimises the halo
    cells of the busiest link (an axis cut in two puts both faces on one link), then the total."""
    D = st.Dim3
    r = st.Radius.constant(0)
    r.set_face(2)
    ML = st.PartitionObjective.MaxLink
    c = D(4, 3, 2)
    # cost of 1x1x8 slabs of 512^3: one 512x512 face (both radii 2: max 2) per link, z cost 2
    assert st.NodePartition.link_cost(D(512, 512, 4096), D(1, 1, 8), r, c) == (512 * 512 * 2 * 2, 512 * 512 * 4 * 2)
    # an axis cut in two: both faces on the one link
    assert st.NodePartition.link_cost(D(512, 512, 1024), D(1, 1, 2), r, c) == (512 * 512 * 4 * 2, 512 * 512 * 4 * 2)
    # stacked cubes -> slabs; a cube of 8 GPUs keeps the reference-like 1x2x4 (busiest link ties 2x2x2, fewer x cuts)
    assert st.NodePartition(D(512, 512, 4096), r, 1, 8, c, ML).dim() == D(1, 1, 8)
    assert st.NodePartition(D(1024, 1024, 1024), r, 1, 8, D(1, 1, 1), ML).dim() == D(1, 2, 4)
    assert st.NodePartition.max_link_dims(D(813, 813, 813), 4, r, c) == D(1, 1, 4)
    # node-level cuts keep the greedy rule; the sub-domains still tile the grid exactly
    p = st.NodePartition(D(600, 600, 900), r, 2, 4, c, ML)
    d = p.dim()
    assert d.x * d.y * d.z == 8
    tot = 0
    for i in range(d.x):
        for j in range(d.y):
            for k in range(d.z):
                s = p.subdomain_size(D(i, j, k))
                tot += s.x * s.y * s.z
    assert tot == 600 * 600 * 900
    # the default objective is the reference's rule
    assert st.NodePartition(D(512, 512, 4096), r, 1, 8, c).dim() == st.NodePartition(D(512, 512, 4096), r, 1, 8, c, st.PartitionObjective.Interface).dim()
