"""Property tests of the halo exchange: random per-direction radius maps (asymmetric, edge- or
corner-only, zero in some directions), random grid sizes, 1-4 sub-domains per process (self-neighbours along axes of
extent 1 or 2 in the decomposition, uneven partitions), random element types and both x layouts, against the
coordinate oracle (stencil2_amd.utils.testing). The reference's own exchange tests fix a handful of patterns and miss
exactly these cases (asymmetric radii on the same-device path, self-neighbours). CPU host backend; the
device variant in tests/test_gpu.py runs a smaller sample on the GPU."""
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as hs

from stencil2_amd.utils.testing import check_exchange, fill_coords

DIRS = [(x, y, z) for z in (-1, 0, 1) for y in (-1, 0, 1) for x in (-1, 0, 1) if (x, y, z) != (0, 0, 0)]


@hs.composite
def exchange_case(draw):
    radii = draw(hs.lists(hs.integers(0, 3), min_size=26, max_size=26))
    n = draw(hs.integers(1, 4))
    # every sub-domain must be at least as wide as the largest halo it feeds: 4 parts of >= 3 cells along any axis
    size = tuple(draw(hs.integers(12, 24)) for _ in range(3))
    dtype = draw(hs.sampled_from([torch.int64, torch.int32, torch.float64]))
    align = draw(hs.booleans())
    return radii, n, size, dtype, align


def _radius(st, radii):
    r = st.Radius.constant(0)
    for (x, y, z), v in zip(DIRS, radii):
        r.set_dir(x, y, z, v)
    return r


def run_case(st, radii, n, size, dtype, align, backend):
    radius = _radius(st, radii)
    dd = st.DistributedDomain(*size, group=st.make_single_group())
    dd.set_backend(backend)
    dd.set_radius(radius)
    dd.set_gpus([0] * n)
    dd.set_x_halo_align(align)
    q = dd.add_data("q", dtype)
    dd.realize()
    bad = 0
    for it in range(2):  # both buffer parities
        fill_coords(dd, q, offset=it)
        dd.exchange()
        bad += check_exchange(dd, q, radius, offset=it)
        dd.swap()
    return bad


@settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(exchange_case())
def test_exchange_random_radius_maps_host(st, case):
    radii, n, size, dtype, align = case
    assert run_case(st, radii, n, size, dtype, align, st.Backend.Host) == 0, case


@pytest.mark.parametrize("seed_radius", [2, 3])
def test_exchange_every_single_direction_host(st, seed_radius):
    """one direction at a time: each of the 26 halos is written alone, exactly where its radius says"""
    for k in range(26):
        radii = [0] * 26
        radii[k] = seed_radius
        assert run_case(st, radii, 2, (14, 13, 12), torch.int64, False, st.Backend.Host) == 0, DIRS[k]
