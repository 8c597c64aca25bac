"""bench.py's control flow on the host backend (--cpu, BASELINE config 1's CPU path): the headline JSON line is
printed BEFORE the transport sweep and again with the sweep (so a transport hanging on real links cannot cost the
headline), a sweep that never returns is abandoned by the deadline with exit 0 behind the headline, and at N > 1 the
warm-up times every transport candidate and keeps the fastest."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")
ARGS = ["--cpu", "--per-gpu", "16", "--steps", "4", "--warmup", "1", "--exchange-iters", "3", "--tune-steps", "2"]


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                        "STENCIL_BENCH_DRY")}
    env["STENCIL_PLAN_FILE"] = "0"
    env["OMP_NUM_THREADS"] = "1"
    env.update(kw)
    return env


def _lines(out):
    return [json.loads(l) for l in out.splitlines() if l.startswith("{")]


def test_headline_printed_before_and_after_sweep():
    r = subprocess.run([sys.executable, BENCH, *ARGS, "--transport-sweep", "on"], env=_env(), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _lines(r.stdout)
    assert len(lines) == 2
    first, second = lines
    assert first["extra"]["transports"] == "pending"
    assert isinstance(second["extra"]["transports"], dict) and "staged" in second["extra"]["transports"]
    assert first["value"] == second["value"] and first["ms_per_step"] == second["ms_per_step"]
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in first
    # the sweep's first line was flushed before the sweep started
    assert r.stdout.index('"pending"') < r.stdout.rindex('"transports": {')


def test_hung_sweep_is_abandoned_behind_the_headline():
    r = subprocess.run([sys.executable, BENCH, *ARGS, "--transport-sweep", "on", "--sweep-deadline", "3"],
                       env=_env(STENCIL_BENCH_SWEEP_HANG="1"), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _lines(r.stdout)
    assert len(lines) == 1 and lines[0]["extra"]["transports"] == "pending"
    assert "abandoning it" in r.stderr


def test_two_ranks_transport_chosen_by_measurement():
    r = subprocess.run([sys.executable, BENCH, *ARGS, "--gpus", "2"], env=_env(), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _lines(r.stdout)
    assert len(lines) == 2  # N > 1: the sweep runs by default
    tt = lines[-1]["config"]["transport_tuned"]
    assert set(tt) == {"colo_uncached", "colo_fine", "colo_coarse", "rccl", "chosen"}
    timed = {k: v["ms"] for k, v in tt.items() if k != "chosen"}
    assert tt["chosen"] == min(timed, key=timed.get)
    tr = lines[-1]["extra"]["transports"]
    assert {"staged", "ref_rule", "astaroth_q8", "peer_store"} <= set(tr)
    assert tr["peer_store"]["devices_used"] >= 1
    assert tr["astaroth_q8"]["halo_bytes"] > tr["ref_rule"]["halo_bytes"]
    assert lines[-1]["n_gpus"] == 2 and lines[-1]["config"]["decomposition"] == "1x1x2"


def test_tune_budget_skips_candidates_and_phases_are_reported():
    """--tune-budget bounds the N > 1 warm-up: with no budget every transport candidate is skipped (agreed over ranks)
    and the model is built with the fixed transports; config.phases_s names every phase that ran, and the reference's
    trimean exchange statistic (bin/bench_exchange.cu:39-63) is reported next to the mean."""
    r = subprocess.run([sys.executable, BENCH, *ARGS, "--gpus", "2", "--tune-budget", "0", "--transport-sweep", "off"],
                       env=_env(), capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = _lines(r.stdout)
    assert len(lines) == 1
    cfg, extra = lines[0]["config"], lines[0]["extra"]
    tt = cfg["transport_tuned"]
    assert all("skipped" in tt[k] for k in ("colo_uncached", "colo_fine", "colo_coarse", "rccl")), tt
    assert tt["chosen"].startswith("fixed")
    for k in ("startup", "transport_warmup", "build", "timed_loop", "exchange_loops"):
        assert k in cfg["phases_s"], cfg["phases_s"]
    assert extra["halo_exchange_trimean_GBps"] is not None and extra["exchange_trimean_ms"] > 0
    assert cfg["tune"]["x3sched"] == 1


def test_tune_switch_sets_stencil_tune_fields():
    r = subprocess.run([sys.executable, BENCH, *ARGS, "--tune", "x3sphw=0.5,nontemporal=0"], env=_env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    t = _lines(r.stdout)[0]["config"]["tune"]
    assert abs(t["x3sphw"] - 0.5) < 1e-6 and t["nontemporal"] is False
