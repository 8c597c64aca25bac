"""Host plans of the fused-triple lockstep schedule (stencil7x3.hip x3_plan, stencil_common.hpp balance_leftover /
lockstep_leftover): the tables the kernel reads must cover every leftover (row group, plane) exactly once, the
second lockstep phase must give every leftover group the same z parts, and the planner's choices for the headline
shapes are pinned. CPU only (the planner is host code); the GPU side is tests/test_gpu.py::test_temporal3_*."""
import collections

import pytest

from stencil2_amd import _C


def _tune(**kw):
    t = _C.StencilTune()
    for k, v in kw.items():
        setattr(t, k, v)
    return t


SHAPES = [(512, 512, 512), (512, 510, 512), (512, 300, 256), (512, 1024, 512), (512, 96, 64), (1024, 512, 128),
          (512, 200, 1000)]


@pytest.mark.parametrize("size", SHAPES)
@pytest.mark.parametrize("jacobi", [True, False])
@pytest.mark.parametrize("left", [0, 1, 2, 3])
def test_leftover_tables_cover_every_plane_once(size, jacobi, left):
    p = _C.stencil7x3_plan(size, jacobi, _tune(x3left=left))
    if p.rounds > 1 or p.parts == 0:
        return
    nz = size[2]
    assert p.parts * p.lockstep_groups == p.blocks and p.lockstep_groups <= p.groups
    if p.zb:  # sphere-weighted parts: parts - 1 nondecreasing bounds inside [0, nz] per group
        for g in range(len(p.zb) // (p.parts - 1)):
            b = p.zb[g * (p.parts - 1):(g + 1) * (p.parts - 1)]
            assert all(0 <= x <= nz for x in b) and b == sorted(b)
    G = p.groups - p.lockstep_groups
    if not p.tabled:
        assert left == 0 or G == 0 or G * nz > 65535
        return
    assert left != 0 and len(p.l0) == len(p.l1) == len(p.odd) == p.blocks
    cover = collections.Counter()
    for a, b in zip(p.l0, p.l1):
        assert 0 <= a <= b <= G * nz
        cover.update(range(a, b))
    assert len(cover) == G * nz and set(cover.values()) == {1}


@pytest.mark.parametrize("size", [(512, 512, 512), (512, 420, 256), (512, 1024, 512)])
def test_lockstep_leftover_parts_are_common_to_every_group(size):
    """x3left 2 with 4 parts (22 / 6 / 107 leftover groups): every block's slice lies in one leftover group, and each z
    range in use is taken by exactly one block of every leftover group (the y-adjacent groups march in step), with
    one direction per z range."""
    p = _C.stencil7x3_plan(size, True, _tune(x3left=2, x3parts=4))
    nz, G = size[2], p.groups - p.lockstep_groups
    assert p.tabled and G > 0
    ranges = collections.defaultdict(list)
    for a, b, o in zip(p.l0, p.l1, p.odd):
        if a == b:
            continue
        g = a // nz
        assert (b - 1) // nz == g, "a lockstep slice stays in one group"
        ranges[(a - g * nz, b - g * nz)].append((g, o))
    for (z0, z1), members in ranges.items():
        assert sorted(g for g, _ in members) == list(range(G)), (z0, z1)
        assert len({o for _, o in members}) == 1
    assert sum(z1 - z0 for z0, z1 in ranges) == nz


def test_headline_plans_are_pinned():
    """512^3 one MI355X (256 resident blocks): Jacobi runs 4 sphere-weighted parts of 64 groups plus the 22 leftover
    groups as a second lockstep phase (profiles/r6/r6ac: 1613-1632 Gcells/s vs 1573-1580 with levelled slices);
    Astaroth 3 parts of 85 groups plus the 2-row group in slices (224.0 vs 241.6 us per triple, profiles/r6/r6ab)."""
    j = _C.stencil7x3_plan((512, 512, 512), True)
    assert (j.parts, j.blocks, j.lockstep_groups, j.groups) == (4, 256, 64, 86) and j.tabled and j.zb
    a = _C.stencil7x3_plan((512, 512, 512), False)
    assert (a.parts, a.blocks, a.lockstep_groups) == (3, 255, 85) and not a.zb
    # equal slices (x3left 0) keep the step-count model's choice and no tables
    e = _C.stencil7x3_plan((512, 512, 512), True, _tune(x3left=0))
    assert not e.tabled and e.parts == 4
    # the estimate prefers the planned leftovers over equal slices
    assert j.steps < e.steps


def test_random_shapes_and_knobs_keep_the_invariants():
    """Random row-group counts, depths, resident-slot counts (CUs left to transports) and knobs: the planned launch
    never exceeds the slots and any table still covers every leftover plane exactly once."""
    import random
    rnd = random.Random(1)
    for _ in range(80):
        size = (512, rnd.randint(3, 1500), rnd.randint(16, 1200))
        jac = rnd.random() < 0.6
        t = _tune(x3left=rnd.choice([0, 1, 2, 3]), x3parts=rnd.choice([0, 0, 0, 2, 3, 4, 5, 8]),
                  x3sphw=rnd.choice([0.0, 0.3, 0.45, 0.6, 1.0]))
        slots = rnd.choice([256, 248, 128, 64, 300])
        p = _C.stencil7x3_plan(size, jac, t, slots)
        if p.rounds > 1 or p.parts == 0:
            continue
        assert p.parts * p.lockstep_groups == p.blocks <= slots
        if p.tabled:
            G, nz = p.groups - p.lockstep_groups, size[2]
            cover = collections.Counter()
            for a, b in zip(p.l0, p.l1):
                assert 0 <= a <= b <= G * nz
                cover.update(range(a, b))
            assert len(cover) == G * nz and set(cover.values()) == {1}
