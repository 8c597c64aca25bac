"""Multi-rank runs over the native TCP process group on the CPU backend (host-staged transport), including fake
multi-node layouts via STENCIL_HOSTNAME (the reference never tested multi-node placement)."""
import os

import pytest

from conftest import run_ranks

WORKER = os.path.join(os.path.dirname(__file__), "mp_worker.py")


def _ok(outs):
    for rc, out in outs:
        assert rc == 0, out[-3000:]


@pytest.mark.parametrize("n,radius,size", [(2, "r1", "12,10,8"), (2, "asym", "13,9,7"), (3, "fec", "15,9,8"),
                                           (4, "r2", "16,12,10")])
def test_staged_exchange_ranks(n, radius, size):
    _ok(run_ranks(n, WORKER, ["exchange", radius, size]))


def test_fake_two_nodes_nodeaware():
    outs = run_ranks(4, WORKER, ["exchange", "r1", "16,12,10"],
                     per_rank_env=lambda r: {"STENCIL_HOSTNAME": f"node{r // 2}"})
    _ok(outs)
    assert all("nodes 2" in out for _, out in outs)


def test_jacobi_ranks_match_oracle():
    _ok(run_ranks(3, WORKER, ["jacobi", "15,11,9"]))


def test_jacobi_eight_ranks_maxlink_slabs():
    """bench.py's 8-GPU layout on the CPU backend: eight ranks over the TCP mesh, MaxLink 1x1x8 slabs (every rank
    exchanges its two z faces with two different ranks, x and y self-periodic), fused pairs vs the torch oracle"""
    outs = run_ranks(8, WORKER, ["jacobi", "12,10,64"],
                     env_extra={"MP_PARTITION": "maxlink", "MP_RANDOM": "1", "MP_TEMPORAL": "2", "MP_AXIS_COST": "4,3,2"})
    _ok(outs)
    assert all("bad 0 " in out and "dim Dim3(1, 1, 8)" in out for _, out in outs)


@pytest.mark.parametrize("n,radius", [(2, "r1"), (3, "fec")])
def test_race_canary_staged(n, radius):
    """NaN-poisoned halos, iteration-tagged interiors, back-to-back exchanges with random transport jitter."""
    _ok(run_ranks(n, WORKER, ["canary", radius, "14,10,9"], env_extra={"MP_JITTER_US": "300"}))


@pytest.mark.parametrize("n", [1, 2, 4])
def test_local_interior_ranks(n):
    """the overlap interior of fused pairs: shrunk only at faces whose halo crosses ranks"""
    _ok(run_ranks(n, WORKER, ["localint", "24,20,18"]))


def test_self_test_ladder_host_backend():
    """realize() with the transport self-test on the host backend (staged over TCP): the probe passes and the
    methods are kept."""
    outs = run_ranks(2, WORKER, ["selftest", "24,20,18"], env_extra={"MP_METHODS": "All"})
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "selftest bad 0" in out and "report [all" not in out, out[-2000:]
        assert ": ok]" in out, out[-2000:]


def test_self_test_one_rank_probe_failure_keeps_ranks_in_step():
    """One rank's first probe throws (TransportOptions.fail_probe_rank) while the other is inside the probe's
    exchange: the probe runs on a forked process group, so the healthy rank times out there, both agree that the
    rung failed, and the ladder goes on to the next rung in step (no desynchronised collectives)."""
    outs = run_ranks(2, WORKER, ["selftest", "24,20,18"],
                     env_extra={"MP_METHODS": "All", "MP_PROBE_FAIL_RANK": "1", "MP_WAIT_TIMEOUT": "3"},
                     timeout=120)
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "selftest bad 0" in out, out[-2000:]
        rep = out.split("report [")[-1].split("]")[0]
        assert rep.split(";")[0].endswith("bad") and rep.rstrip().endswith(": ok"), rep
