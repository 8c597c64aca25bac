"""GPU: bounded RCCL communicator creation and bench.py's multi-section output on one MI355X.

* A rank stuck before RCCL creation (TransportOptions.stall_rccl_init_rank) costs the wait timeout, not a hang: the
  non-blocking creation is abandoned, every RCCL channel falls back to host-staged, and the halos are still exact.
* bench.py prints its headline before the transport sweep and again after it; an RCCL entry whose communicator never
  forms records an error and the run still ends with exit 0; the with-exchange figure (config 2 as defined) and the
  single-process PeerCopy / config-4 Astaroth entries are present.
"""
import json
import os
import subprocess
import sys
import time

import pytest

from stencil2_amd.utils.testing import check_exchange, fill_coords

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_init_stall_is_bounded_and_falls_back(st):
    import torch

    tr = st.TransportOptions()
    tr.stall_rccl_init_rank = 0
    tr.wait_timeout = 3.0
    dd = st.DistributedDomain(19, 13, 11, group=st.make_single_group())
    dd.set_backend(st.Backend.Device)
    dd.set_transport_options(tr)
    r = st.Radius.constant(1)
    dd.set_radius(r)
    dd.set_gpus([0, 0])
    dd.set_methods(st.MethodFlags.Rccl)
    q = dd.add_data("c", torch.int64)
    t0 = time.monotonic()
    dd.realize()
    assert time.monotonic() - t0 < 30
    assert "timed out" in dd.rccl_status()
    assert dd.exchange_bytes_for_method(st.MethodFlags.Rccl) == 0
    assert dd.exchange_bytes_for_method(st.MethodFlags.Staged) > 0
    for _ in range(2):
        fill_coords(dd, q)
        dd.exchange()
        assert check_exchange(dd, q, r) == 0
        dd.swap()


def test_rccl_nonblocking_loopback_status(st):
    import torch

    dd = st.DistributedDomain(19, 13, 11, group=st.make_single_group())
    dd.set_backend(st.Backend.Device)
    r = st.Radius.constant(2)
    dd.set_radius(r)
    dd.set_gpus([0, 0])
    dd.set_methods(st.MethodFlags.Rccl)
    q = dd.add_data("c", torch.int64)
    dd.realize()
    assert dd.rccl_status() == "ok"
    assert dd.exchange_bytes_for_method(st.MethodFlags.Rccl) > 0
    for _ in range(3):
        fill_coords(dd, q)
        dd.exchange()
        assert check_exchange(dd, q, r) == 0
        dd.swap()


def test_bench_two_lines_and_stalled_rccl_entry():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["STENCIL_RCCL_STALL_RANK"] = "0"
    env["STENCIL_PLAN_FILE"] = "0"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--per-gpu", "128", "--steps", "4",
                        "--warmup", "2", "--exchange-iters", "4", "--transport-sweep", "on"],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 2, r.stdout
    assert lines[0]["extra"]["transports"] == "pending" and lines[0]["value"] == lines[1]["value"]
    assert lines[0]["extra"]["gcells_with_exchange"] > 0  # config 2 as defined: every halo copied
    tr = lines[1]["extra"]["transports"]
    assert "error" in tr["rccl"] and "RCCL" in tr["rccl"]["error"], tr["rccl"]
    assert tr["peer_store"]["devices_used"] == 1 and "GBps" in tr["peer_store"], tr["peer_store"]
    assert "GBps" in tr["peer_engine"], tr["peer_engine"]
    assert tr["astaroth_q8"]["decomposition"] == "1x1x1" and tr["astaroth_q8"]["GBps"] > 0


def test_bench_triple_schedule_phase():
    """The driver's command (512^3, fused triples): the schedule phase times every candidate (sphere weight x leftover
    plan), keeps one of them, records the times and its wall time; --schedule-rounds 0 skips it."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["STENCIL_PLAN_FILE"] = "0"
    base = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "20", "--warmup", "5", "--exchange-iters", "4",
            "--transport-sweep", "off", "--with-exchange", "off"]
    r = subprocess.run(base, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    d = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")][-1]
    s = d["config"]["schedule_tuned"]
    times = {k: v for k, v in s.items() if k.endswith("_ms")}
    assert len(times) == 5 and all(v > 0 for v in times.values())
    assert f"sphw{s['x3sphw']}_left{s['x3left']}_ms" in times and d["config"]["tune"]["x3left"] == s["x3left"]
    assert d["config"]["phases_s"]["schedule_warmup"] > 0 and d["value"] > 0
    r = subprocess.run(base + ["--schedule-rounds", "0"], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    d = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")][-1]
    assert d["config"]["schedule_tuned"] is None and "schedule_warmup" not in d["config"]["phases_s"]
