"""bench.py's weak-scaling grids: exact 512^3 per GPU (default) and the reference's cbrt cube."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _check_cubes(st, g, n, objective):
    r = st.Radius.constant(0)
    r.set_face(1)
    p = st.NodePartition(st.Dim3(*g), r, 1, n, st.Dim3(4, 3, 2), objective)
    d = p.dim()
    assert d.x * d.y * d.z == n
    for i in range(d.x):
        for j in range(d.y):
            for k in range(d.z):
                assert p.subdomain_size(st.Dim3(i, j, k)) == st.Dim3(512, 512, 512)
    return d


@pytest.mark.parametrize("n,want", [(1, (512, 512, 512)), (2, (512, 512, 1024)), (4, (512, 1024, 1024)),
                                    (8, (512, 1024, 2048))])
def test_exact_grid_interface_cuts(st, n, want):
    g = bench.weak_grid(st, 512, n, "exact", (4, 3, 2), st.PartitionObjective.Interface)
    assert g == want
    _check_cubes(st, g, n, st.PartitionObjective.Interface)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 6, 8])
def test_exact_grid_max_link_is_z_slabs(st, n):
    """bench.py's default: on a fully connected xGMI node the busiest link decides, so n cubes stack along z
    (two faces per GPU, one per link; x and y wrap in the stencil kernel)."""
    g = bench.weak_grid(st, 512, n, "exact", (4, 3, 2), st.PartitionObjective.MaxLink)
    assert g == (512, 512, 512 * n)
    d = _check_cubes(st, g, n, st.PartitionObjective.MaxLink)
    assert (d.x, d.y, d.z) == (1, 1, n)


def test_exact_grid_reference_costs_is_a_cube_at_8(st):
    # the reference's equal cut costs decompose 8 GPUs 2x2x2: the exact grid is then the cbrt cube itself
    assert bench.weak_grid(st, 512, 8, "exact", (1, 1, 1), st.PartitionObjective.Interface) == (1024, 1024, 1024)


@pytest.mark.parametrize("n,side", [(1, 512), (2, 645), (4, 813), (8, 1024)])
def test_cbrt_grid_is_the_reference_rule(st, n, side):
    for obj in (st.PartitionObjective.MaxLink, st.PartitionObjective.Interface):
        assert bench.weak_grid(st, 512, n, "cbrt", (4, 3, 2), obj) == (side, side, side)
