#!/usr/bin/env python3
"""Headline benchmark: Jacobi3D weak scaling, 512^3 cells per GPU, fp32, one process per GPU.

Metric (BASELINE.json): "halo-exchange GB/s + Jacobi3D Gcells/s, 512^3/GPU weak scaling at 1/2/4/8 MI355X".
`value` is the whole-job Jacobi3D throughput in Gcells/s (global cells x steps / time). One step is the
reference's full iteration (bin/jacobi3d.cu:265-346): interior stencil overlapped with the halo exchange of all
faces (periodic), exterior stencil, swap. Every GPU holds exactly 512^3 cells (--grid exact); the decomposition is
the NodeAware partitioner's MaxLink choice for the xGMI mesh (1x1xN slabs: two faces per GPU, each on its own
link); --grid cbrt runs the reference's cube rule (512 * N^0.33333 per axis: 645/813/1024 for N=2/4/8) and
--partition interface the reference's cut rule.
Secondary numbers in the JSON line: the halo-exchange GB/s of an exchange-only loop on the same decomposition
(bin/bench_exchange.cu definition: aggregate halo bytes / time).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
  N>1 runs one rank per GPU. Under torch.distributed.run (WORLD_SIZE set) it must equal WORLD_SIZE; without a
  launcher, bench.py itself spawns N fresh child ranks (stencil2_amd/launch.py, loaded by path) before importing
  torch or touching the GPU, waits for them with a bounded timeout, stops every sibling when one fails and exits with
  the failing rank's code. Rank 0 prints the JSON line (reference: one rank per GPU from the job script,
  scripts/summit/weak_256n.sh:26-30).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time


def weak_grid(st, per_gpu: int, n: int, rule: str, axis_cost, objective) -> tuple:
    """Global grid of the weak-scaling run on n GPUs.

    cbrt: the reference's cube of side per_gpu * n^(1/3) (bin/jacobi3d.cu:167-169).
    exact: every sub-domain exactly per_gpu^3, so per-GPU work is the N=1 work to the cell; the decomposition d is
    the partitioner's choice for n cubes (MaxLink on the node's xGMI mesh: 1x1xN slabs, two faces per GPU on two
    links; Interface: the reference's greedy cut of the cbrt-scaled cube, 1x1x2 / 1x2x2 / 1x2x4), the grid is
    per_gpu x d.
    """
    L = st.models.weak_scaled_size(per_gpu, n)
    if rule == "cbrt" or n == 1:
        return (L, L, L)
    r = st.Radius.constant(0)
    r.set_face(1)
    cost = st.Dim3(*axis_cost)
    if objective == st.PartitionObjective.MaxLink:
        # every factorization d of n, scored on the grid of n per_gpu^3 cubes it forms (busiest link, total)
        best = None
        for dx in range(1, n + 1):
            for dy in range(1, n // dx + 1):
                if n % (dx * dy):
                    continue
                dz = n // (dx * dy)
                g = st.Dim3(per_gpu * dx, per_gpu * dy, per_gpu * dz)
                c = st.NodePartition.link_cost(g, st.Dim3(dx, dy, dz), r, cost)
                key = (c, dx, dy)
                if best is None or key < best[0]:
                    best = (key, st.Dim3(dx, dy, dz))
        d = best[1]
    else:
        d = st.NodePartition(st.Dim3(L, L, L), r, 1, n, cost).dim()
    grid = (per_gpu * d.x, per_gpu * d.y, per_gpu * d.z)
    p = st.NodePartition(st.Dim3(*grid), r, 1, n, cost, objective)
    if p.dim() != d or any(p.subdomain_size(st.Dim3(i, j, k)) != st.Dim3(per_gpu, per_gpu, per_gpu)
                           for i in range(d.x) for j in range(d.y) for k in range(d.z)):
        return (L, L, L)  # the partitioner would not cut the scaled grid into equal cubes: the reference rule
    return grid


def transport_sweep(st, torch, dist, args, world, device, red_dev, axis_cost, objective, topt_base):
    """Exchange-only GB/s of the headline decomposition with each transport set in turn, plus the reference-rule
    point (the cbrt cube cut by the reference's greedy Interface rule with equal axis costs: 2x2x2 at N = 8, the
    bench_exchange --x 1024 --y 1024 --z 1024 --fr 2 config), so one multi-GPU run yields the whole ladder
    (reference: src/stencil.cu:163-194 method ladder; scripts/summit/weak_256n.sh:26-30 per-method sweeps).

    Radius-2 faces, one fp32 quantity (the depth-2 exchange of a fused pair), blocking exchange()+swap() as in
    bin/bench_exchange.cu:39-63 and the same exchanges stream-ordered. Each entry realizes its own domain on a fresh
    native process group with a short timeout, so a transport that fails on one rank costs that entry (an "error"
    string), not the run. The number of timed exchanges is agreed over ranks from a timed probe exchange, and the
    whole section stops starting entries after --sweep-budget seconds."""
    M = st.MethodFlags
    C = st.TransportOptions.Completion
    sets = [("colo_store", M.Colocated | M.Kernel, "store", C.Kernel),
            ("colo_engine", M.Colocated | M.Kernel, "engine", C.Kernel),
            ("colo_ipcevent", M.Colocated | M.Kernel, "store", C.IpcEvent),
            ("rccl", M.Rccl | M.Kernel, "store", C.Kernel), ("staged", M.Staged | M.Kernel, "store", C.Kernel),
            ("ref_rule", M.All, "store", C.Kernel)]
    out = {}
    t_start = time.perf_counter()

    def agreed_max(v):
        t = torch.tensor([float(v)], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    for name, m, copy, completion in sets:
        if agreed_max(time.perf_counter() - t_start) > args.sweep_budget:
            out[name] = {"skipped": f"sweep budget {args.sweep_budget:.0f} s spent"}
            continue
        rec = {}
        ok = 1.0
        dd = None
        if int(os.environ.get("RANK", "0")) == 0:
            print(f"[bench] transport {name}: starting", file=sys.stderr, flush=True)
        try:
            if name == "ref_rule":
                L = st.models.weak_scaled_size(args.per_gpu, world)
                g, obj, cost = (L, L, L), st.PartitionObjective.Interface, (1, 1, 1)
            else:
                g, obj, cost = weak_grid(st, args.per_gpu, world, args.grid, axis_cost, objective), objective, axis_cost
            grp = st.init_process_group(set_default=False, timeout_s=15.0)
            dd = st.DistributedDomain(*g, group=grp)
            r = st.Radius.constant(0)
            r.set_face(2)
            dd.set_radius(r)
            dd.add_data("q", torch.float32)
            dd.set_methods(m)
            dd.set_gpus([device])
            dd.set_axis_cost(st.Dim3(*cost))
            dd.set_partition_objective(obj)
            dd.set_plan_file("")
            dd.set_x_halo_align(bool(args.x_halo_align))
            dd.set_interior_align(args.interior_align)
            topt = st.TransportOptions()
            topt.inbox = topt_base.inbox
            topt.completion = completion
            topt.fuse_flags = topt_base.fuse_flags
            topt.colo_copy = topt.Copy.Engine if copy == "engine" else topt.Copy.Store
            topt.wait_timeout = 10.0  # a failing entry gives up within seconds, not minutes
            dd.set_transport_options(topt)
            dd.realize()
            pd = dd.placement_dim()
            rec["grid"] = list(g)
            rec["decomposition"] = f"{pd.x}x{pd.y}x{pd.z}"
            rec["asked"] = st.methods_to_string(m)
            rec["realized"] = st.methods_to_string(dd.methods())
            rec["bytes_by_method"] = {st.methods_to_string(f): int(dd.exchange_bytes_for_method(f))
                                      for f in (M.Kernel, M.PeerCopy, M.Colocated, M.Rccl, M.Staged)
                                      if dd.exchange_bytes_for_method(f) > 0}
            xbytes = dd.exchange_bytes_for_method(M.All)
            for _ in range(2):
                dd.exchange()
                dd.swap()
            torch.cuda.synchronize()
            t = time.perf_counter()
            dd.exchange()
            dd.swap()
            probe = agreed_max(time.perf_counter() - t)
            iters = int(max(1, min(args.exchange_iters, 1.0 / max(probe, 1e-6))))
            colo = dd.exchange_bytes_for_method(M.Colocated) > 0 and completion != C.StreamOp
            if colo:
                dd.set_transport_log(iters)
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            t = time.perf_counter()
            for _ in range(iters):
                dd.exchange()
                dd.swap()
            el = agreed_max(time.perf_counter() - t)
            if colo:
                rec["colo_kernels_us"] = colo_breakdown(dd.transport_log(0))
                dd.set_transport_log(0)
            xs = torch.cuda.Stream()
            dd.exchange_async(xs.cuda_stream, 0)
            dd.swap()
            xs.synchronize()
            dd.sync_exchange()
            if world > 1:
                dist.barrier()
            t = time.perf_counter()
            for _ in range(iters):
                dd.exchange_async(xs.cuda_stream, 0)
                dd.swap()
            xs.synchronize()
            dd.sync_exchange()
            el2 = agreed_max(time.perf_counter() - t)
            rec.update({"iters": iters, "halo_bytes": int(xbytes), "exchange_ms": round(el / iters * 1e3, 4),
                        "GBps": round(xbytes * iters / el / 1e9, 3),
                        "stream_GBps": round(xbytes * iters / el2 / 1e9, 3)})
        except Exception as e:  # noqa: BLE001 -- one transport failing must not end the run
            ok = 0.0
            rec["error"] = f"{type(e).__name__}: {str(e)[:300]}"
        del dd
        if agreed_max(1.0 - ok) > 0 and "error" not in rec:
            rec["error"] = "failed on another rank"
        out[name] = rec
        if int(os.environ.get("RANK", "0")) == 0:
            print(f"[bench] transport {name}: {rec}", file=sys.stderr, flush=True)
    return out


def colo_breakdown(log) -> dict:
    """Median phases (us) of the fused co-located transport kernels from DistributedDomain.transport_log: per
    exchange {send start, after the credit wait, after the copies, signal, recv start, after the arrival wait, after
    the copies, signal} in 100-MHz ticks (0: that kernel did not run / that phase does not exist)."""
    import statistics

    def med(vals):
        vals = [v for v in vals if v is not None and v >= 0]
        return round(statistics.median(vals) / 100.0, 2) if vals else None

    def ph(e, a, b):
        return e[b] - e[a] if e[a] and e[b] else None

    return {"send_wait": med([ph(e, 0, 1) for e in log]), "send_copy": med([ph(e, 1, 2) for e in log]),
            "send_signal": med([ph(e, 2, 3) for e in log]), "recv_wait": med([ph(e, 4, 5) for e in log]),
            "recv_copy": med([ph(e, 5, 6) for e in log]), "recv_signal": med([ph(e, 6, 7) for e in log]),
            "send_end_to_recv_start": med([ph(e, 3, 4) for e in log]), "exchanges": len(log)}


def _gpus_sysfs() -> int:
    """GPUs of this node from the KFD topology (no HIP call: the HIP runtime must not start before the queue limit
    below is set)."""
    import glob
    n = 0
    for f in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id"):
        try:
            n += int(open(f).read().strip() or 0) != 0
        except (OSError, ValueError):
            pass
    return n


def _limit_queues_when_sharing():
    """Ranks sharing one GPU (a rehearsal of the multi-GPU run on a smaller box): keep ranks x hardware queues per
    process <= 8. Beyond that the GPU time-slices the processes' queues and every cross-process hand-off waits a
    scheduling quantum: one MI355X, 8 ranks x 128^3, 39.3 / 6.0 / 2.0 ms per step with 4 / 2 / 1 queues per
    process, 4 ranks 12.4 vs 0.30 ms with 4 vs 2 (profiles/r3/cliff/). One process per GPU is left alone."""
    local = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    ngpu = _gpus_sysfs()
    if ngpu and local > ngpu and "GPU_MAX_HW_QUEUES" not in os.environ:
        per_gpu = -(-local // ngpu)
        os.environ["GPU_MAX_HW_QUEUES"] = str(max(1, 8 // per_gpu))


def _launcher():
    """stencil2_amd/launch.py without importing the package (its __init__ imports torch and the HIP runtime)."""
    import importlib.util
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "stencil2_amd", "launch.py")
    spec = importlib.util.spec_from_file_location("_stencil2_launch", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def rank_setup(gpus: int, launch_timeout: float, argv: list[str]):
    """None: this process is a rank (run the bench). An int: the exit code of this process (a spawning parent, or a
    --gpus / WORLD_SIZE mismatch). Runs before torch is imported: no HIP call may precede the fork."""
    world = os.environ.get("WORLD_SIZE")
    if world is None:
        if gpus <= 1:
            return None
        return _launcher().spawn_ranks([sys.executable, os.path.abspath(__file__), *argv], gpus,
                                       timeout=launch_timeout if launch_timeout > 0 else None)
    if int(world) != gpus:
        print(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: the launcher and the bench disagree on the number "
              f"of GPUs; refusing to time a different job than the one asked for", file=sys.stderr, flush=True)
        return 2
    if os.environ.get("STENCIL_BENCH_DRY"):  # launcher tests (CPU): report the rank layout, touch nothing else
        rank = int(os.environ.get("RANK", "0"))
        if os.environ.get("STENCIL_BENCH_DRY_FAIL_RANK") == str(rank):
            return 3
        if os.environ.get("STENCIL_BENCH_DRY_SLEEP"):
            time.sleep(float(os.environ["STENCIL_BENCH_DRY_SLEEP"]))
        print(json.dumps({"rank": rank, "world": int(world), "local_rank": int(os.environ.get("LOCAL_RANK", "-1")),
                          "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}",
                          "torch_loaded": "torch" in sys.modules}), flush=True)
        return 0
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--per-gpu", type=int, default=512)
    ap.add_argument("--exchange-iters", type=int, default=20)
    ap.add_argument("--no-overlap", action="store_true")
    ap.add_argument("--methods", default="all")
    ap.add_argument("--nt", type=int, default=1, help="non-temporal stencil stores")
    ap.add_argument("--altz", type=int, default=1,
                    help="alternate the z-march direction every pair (128-B-aligned rows: 1276-1290 with vs 1256-1272 "
                         "Gcells/s without, profiles/r4/q)")
    ap.add_argument("--ty", type=int, default=2, help="rows per lane of the stencil kernel (2/4/8)")
    ap.add_argument("--variant", type=int, default=2,
                    help="single-step kernel variant (2: VALU LDS z-march, 8: MFMA x-line update; needs --temporal 1)")
    ap.add_argument("--nw", type=int, default=8, help="waves per block of the stencil kernel")
    ap.add_argument("--x2nw", type=int, default=12, help="waves per block of the fused two-step kernel (8/12/16)")
    ap.add_argument("--x2pf", type=int, default=1, help="planes of z lookahead of the fused two-step kernel (1/2/3)")
    ap.add_argument("--x2row", type=int, default=1,
                    help="fused pairs: one wave per whole 512-cell row when x wraps in-kernel (fp32); 0 = columns")
    ap.add_argument("--x2reserve", type=int, default=8,
                    help="overlapped fused pairs: CUs the interior sweep leaves to the transport kernels")
    ap.add_argument("--zchunk", type=int, default=0, help="z planes per block (0 = auto)")
    ap.add_argument("--x2sched", type=int, default=1,
                    help="fused-pair work split: 1 = balanced segments over the resident blocks, 0 = fixed z-chunks")
    ap.add_argument("--temporal", type=int, default=2,
                    help="steps fused per sweep: 2 = temporal blocking (one depth-2 halo exchange + one fused "
                         "S(S(u)) sweep per two steps, bitwise equal to single steps), 1 = one exchange + sweep per step")
    ap.add_argument("--x2xfast", type=int, default=0, help="fused-pair column order: 1 x-major, 0 y-major")
    ap.add_argument("--wrap", type=int, default=1,
                    help="fused pairs read the periodic image along axes the decomposition leaves whole (no self-copy "
                         "of those halos); 0 = copy every halo")
    ap.add_argument("--x-halo-align", type=int, default=0,
                    help="x halos inside the interior's first / last 64-B sector (LocalDomain::set_x_halo_align): "
                         "one sector per row end for x-face copies; every row spans one more sector")
    ap.add_argument("--x-face-lines", type=int, default=0,
                    help="same-GPU x-face copies as whole 128-B lines (TransportOptions.x_face_sectors)")
    ap.add_argument("--interior-align", type=int, default=128, choices=[64, 128],
                    help="byte alignment of every row's first interior cell: 128 = whole L2 lines per 512-cell row "
                         "(1150-1194 -> 1285-1287 Gcells/s on one MI355X, profiles/r4/i/), 64 = one sector (r1-r3)")
    ap.add_argument("--axis-cost", default="4,3,2",
                    help="NodeAware partition cost per interface cell of x,y,z cuts (1,1,1 = the reference's rule)")
    ap.add_argument("--partition", choices=["maxlink", "interface"], default="maxlink",
                    help="NodeAware cut rule inside the node: maxlink = fewest halo cells on the busiest xGMI link "
                         "(then fewest in total): 1x1xN slabs of 512^3; interface = the reference's greedy minimum "
                         "interface (1x2x2 / 1x2x4)")
    ap.add_argument("--grid", choices=["exact", "cbrt"], default="exact",
                    help="weak-scaling grid: exact = every GPU holds exactly per_gpu^3 cells (global grid = per_gpu x the "
                         "decomposition of the cbrt-scaled cube); cbrt = the reference's rule, a per_gpu*N^(1/3) cube "
                         "(bin/jacobi3d.cu:167-169: 645^3 / 813^3 / 1024^3 at N = 2 / 4 / 8, ragged sub-domains)")
    ap.add_argument("--overlap", choices=["auto", "on", "off"], default="auto",
                    help="interior/exchange/exterior overlap (auto: only when some halo leaves the GPU, and then "
                         "overlapped or whole-region pairs, whichever runs faster in the warm-up)")
    ap.add_argument("--colo-copy", choices=["auto", "store", "engine"], default="store",
                    help="co-located (HIP IPC) halos: the pack kernel stores into the peer's inbox (store, default), or "
                         "a DMA engine copies the packed message (engine); auto: both tried in the warm-up. Engine "
                         "copies never won on one MI355X and, with 4 ranks sharing it, ran at 0.6-1.7 s per step and "
                         "left the store path 3.5x slower afterwards (profiles/r3/check4), so they are opt-in")
    ap.add_argument("--inbox", choices=["uncached", "fine", "coarse"], default="uncached",
                    help="memory of the co-located receive slots (TransportOptions.inbox)")
    ap.add_argument("--completion", choices=["kernel", "streamop", "ipcevent"], default="kernel",
                    help="co-located arrival/credit signalling: bounded spin kernels, hipStreamWait/WriteValue64, or "
                         "interprocess events with host notify/ack (the reference's design)")
    ap.add_argument("--fuse-flags", type=int, default=1,
                    help="co-located flag waits/signals folded into the pack/unpack kernels (0: separate kernels)")
    ap.add_argument("--self-test", type=int, default=1,
                    help="multi-process: verify the transports on a probe domain first and fall back along "
                         "Colocated -> Rccl -> Staged until every halo arrives correctly")
    ap.add_argument("--tune-steps", type=int, default=8,
                    help="steps per timed round of the overlap choice (auto, remote halos only; 0 = no choice)")
    ap.add_argument("--transport-sweep", choices=["auto", "on", "off"], default="auto",
                    help="after the headline: exchange-only GB/s of every transport set on the same decomposition "
                         "and of the reference-rule cube (auto: only with N > 1)")
    ap.add_argument("--sweep-budget", type=float, default=30.0,
                    help="seconds after which the transport sweep starts no further entry")
    ap.add_argument("--launch-timeout", type=float, default=3000,
                    help="--gpus N>1 without a launcher: seconds before the spawned ranks are stopped (0 = none)")
    args = ap.parse_args()
    rc = rank_setup(args.gpus, args.launch_timeout, sys.argv[1:])
    if rc is not None:
        return rc
    _limit_queues_when_sharing()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    device = local_rank % max(1, ndev)
    torch.cuda.set_device(device)
    # one rank per GPU: RCCL for the harness barrier/max-reduce. More ranks than GPUs (a rehearsal on a 1-GPU box,
    # ranks sharing the device through HIP IPC) cannot use RCCL, so the harness collectives go over gloo.
    shared = world > ndev
    if world > 1:
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
    red_dev = "cpu" if shared else "cuda"

    import stencil2_amd as st

    pg = st.init_process_group()
    n = world
    L = st.models.weak_scaled_size(args.per_gpu, n)
    axis_cost = tuple(int(v) for v in args.axis_cost.split(","))
    objective = st.PartitionObjective.MaxLink if args.partition == "maxlink" else st.PartitionObjective.Interface
    grid = weak_grid(st, args.per_gpu, n, args.grid, axis_cost, objective)
    methods = st.MethodFlags.All
    if args.methods != "all":
        methods = st.MethodFlags.None_
        for m in args.methods.split(","):
            methods = methods | getattr(st.MethodFlags, {"staged": "Staged", "rccl": "Rccl", "colo": "Colocated",
                                                          "peer": "PeerCopy", "kernel": "Kernel"}[m])

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    # Transport self-test (multi-process only, DistributedDomain::set_self_test, run inside realize): a
    # coordinate-encoded field on a small probe domain with the model's radius, placement and transports is exchanged
    # and checked cell by cell on every rank; any wrong halo or error drops Colocated, then Rccl (host-staged), so a
    # scaling run never times silently corrupted halos. An RCCL communicator that fails to form falls back to the
    # host-staged path on every rank as well.
    topt = st.TransportOptions()
    topt.inbox = {"uncached": topt.Inbox.Uncached, "fine": topt.Inbox.Fine, "coarse": topt.Inbox.Coarse}[args.inbox]
    topt.colo_copy = topt.Copy.Engine if args.colo_copy == "engine" else topt.Copy.Store
    topt.completion = {"kernel": topt.Completion.Kernel, "streamop": topt.Completion.StreamOp,
                       "ipcevent": topt.Completion.IpcEvent}[args.completion]
    topt.fuse_flags = bool(args.fuse_flags)
    topt.x_face_sectors = bool(args.x_face_lines)
    if os.environ.get("STENCIL_PREFLIGHT_FORCE_FAIL"):  # rehearses the fallback (scripts): IPC probe reports failure
        topt.fail_ipc_probe = True

    tune = st.StencilTune()
    tune.nontemporal = bool(args.nt)
    tune.alternate_z = bool(args.altz)
    tune.ty = args.ty
    tune.nw = args.nw
    tune.variant = args.variant
    tune.x2nw = args.x2nw
    tune.x2pf = args.x2pf
    tune.x2row = args.x2row
    tune.zchunk = args.zchunk
    tune.x2reserve = args.x2reserve
    tune.x2sched = args.x2sched
    tune.x2xfast = args.x2xfast
    overlap = not args.no_overlap and args.overlap != "off"
    model = st.Jacobi3D(grid, gpus=[device], methods=methods, overlap=overlap,
                        auto_overlap=args.overlap == "auto", tune=tune, temporal=args.temporal, group=pg,
                        axis_cost=axis_cost, partition=objective, wrap_self=bool(args.wrap), transport=topt,
                        self_test=bool(args.self_test) and world > 1, x_halo_align=bool(args.x_halo_align),
                        interior_align=args.interior_align)
    model.init()
    methods = model.domain.methods()
    preflight = model.domain.self_test_report() or "skipped"
    colo = model.domain.exchange_bytes_for_method(st.MethodFlags.Colocated) > 0
    model.prepare()  # hipGraph capture + instantiation (no steps run) outside the timed region
    model.run(args.warmup)
    model.synchronize()
    barrier()
    # overlapped vs whole-region pairs (remote halos only): both run, the faster one (max over ranks, best of two
    # rounds) is kept for the timed loop -- part of the warm-up, every rank takes the same decision
    overlap_tuned = None
    if args.overlap == "auto" and args.tune_steps > 0 and model.can_toggle_overlap():
        def timed_run(k):
            barrier()
            t = time.perf_counter()
            model.run(k)
            model.synchronize()
            dt = torch.tensor([time.perf_counter() - t], dtype=torch.float64, device=red_dev)
            if world > 1:
                dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            return float(dt.item()) / k * 1e3
        best = {}
        k = max(2, args.tune_steps // 2 * 2)
        r0 = args.x2reserve
        # (mode, CUs left to the transports, co-located copy): mode 1 = slabs beside the sweep, 2 = slabs after
        # it, 0 = whole-region pairs, 3 = pipelined whole-region pairs; copy "s" = pack kernel stores into the peer inbox, "e" = DMA engine copy (the
        # transports then need fewer CUs: also tried with a quarter of the reserve)
        copies = ["s", "e"] if colo and args.colo_copy == "auto" else ["e" if args.colo_copy == "engine" else "s"]
        cands = []
        for cp in copies:
            # mode 3 (pipelined pairs: the next exchange gated on the sweep's published boundary planes) needs the
            # pack-kernel stores
            if cp == "s" and model.can_pipeline():
                cands += [(3, r0, cp), (3, max(1, r0 // 2), cp), (3, 2 * r0, cp)]
            cands += [(1, r0, cp), (1, max(1, r0 // 2), cp), (1, 2 * r0, cp), (2, r0, cp), (0, r0, cp)]
            if cp == "e":
                cands.append((1, max(1, r0 // 4), cp))

        def apply(c):
            model.domain.set_colo_copy(topt.Copy.Engine if c[2] == "e" else topt.Copy.Store)
            model.set_overlap_mode(c[0])
            model.set_comm_reserve(c[1])

        skip = set()
        for c in cands + cands:
            if c in skip:
                continue
            apply(c)
            model.run(2)
            model.synchronize()
            # a 2-step probe first: a candidate far slower than the best so far (ranks sharing one GPU: DMA-engine
            # copies beside overlapped sweeps ran at ~0.8 s per step, profiles/r3/check2) is not given full rounds
            ref = min(best.values(), default=float("inf"))
            t = timed_run(2)
            if t > 4 * ref:
                skip.add(c)
                best[c] = min(best.get(c, float("inf")), t)
            else:
                best[c] = min(best.get(c, float("inf")), t, timed_run(k))
            if rank == 0:
                print(f"[bench] overlap choice {c}: {best[c]:.4f} ms/step{' (skipped)' if c in skip else ''}",
                      file=sys.stderr, flush=True)
        choice = min(cands, key=lambda c: best[c])
        apply(choice)
        model.run(2)
        model.synchronize()
        barrier()
        overlap_tuned = {"mode": choice[0], "reserve": choice[1], "colo_copy": "engine" if choice[2] == "e" else "store",
                         **{f"m{c[0]}_r{c[1]}_{c[2]}_ms": round(best[c], 4) for c in cands}}
    t0 = time.perf_counter()
    model.run(args.steps)  # every step is enqueued; whole blocks of steps replay as one hipGraph where possible
    model.synchronize()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
    t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    cells = grid[0] * grid[1] * grid[2]
    gcells = cells * args.steps / elapsed / 1e9

    # exchange-only loop on the same decomposition (halo-exchange GB/s, bench_exchange definition)
    dd = model.domain
    dd.set_comm_max_blocks(0)  # the exchange alone may use the whole GPU (the overlapped steps confine it to 8 CUs)
    xbytes = dd.exchange_bytes_for_method(st.MethodFlags.All)
    for _ in range(3):  # untimed: the first full exchanges after wrapped pairs touch cold halo lines
        dd.exchange()
        dd.swap()
    colo_log = colo and topt.completion != topt.Completion.StreamOp
    if colo_log:  # device timestamps of the fused co-located kernels (wait vs copy), no host cost
        dd.set_transport_log(args.exchange_iters)
    barrier()
    t1 = time.perf_counter()
    for _ in range(args.exchange_iters):
        dd.exchange()
        dd.swap()
    torch.cuda.synchronize()
    xel = time.perf_counter() - t1
    colo_phases = colo_breakdown(dd.transport_log(0)) if colo_log else None
    if colo_log:
        dd.set_transport_log(0)
    tx = torch.tensor([xel], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(tx, op=dist.ReduceOp.MAX)
    xel = float(tx.item())
    xgbs = xbytes * args.exchange_iters / xel / 1e9
    # the same exchanges stream-ordered back to back (exchange_async on one stream, a single synchronize at the end):
    # the transports' own rate without the host round trip of every blocking exchange()
    xs = torch.cuda.Stream()
    for _ in range(3):  # untimed: the first launches on a new stream create its hardware queue (~ms)
        dd.exchange_async(xs.cuda_stream, 0)
        dd.swap()
    xs.synchronize()
    dd.sync_exchange()
    barrier()
    t2 = time.perf_counter()
    for _ in range(args.exchange_iters):
        dd.exchange_async(xs.cuda_stream, 0)
        dd.swap()
    xs.synchronize()
    dd.sync_exchange()
    xel2 = time.perf_counter() - t2
    tx2 = torch.tensor([xel2], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(tx2, op=dist.ReduceOp.MAX)
    xgbs_stream = xbytes * args.exchange_iters / float(tx2.item()) / 1e9

    pdim = model.domain.placement_dim()
    model_cfg = {
        "decomposition": f"{pdim.x}x{pdim.y}x{pdim.z}", "methods": st.methods_to_string(methods), "preflight": preflight,
        "overlap": model.overlapping(), "overlap_mode": model.overlap_mode(), "overlap_tuned": overlap_tuned,
        "x_halo_align": bool(args.x_halo_align), "interior_align": args.interior_align,
        "x_face_lines": bool(args.x_face_lines),
        "nontemporal": bool(args.nt), "alternate_z": bool(args.altz), "ty": args.ty, "nw": args.nw,
        "variant": args.variant, "x2nw": args.x2nw, "x2pf": args.x2pf, "x2row": args.x2row, "x2sched": args.x2sched,
        "x2xfast": args.x2xfast, "zchunk": args.zchunk, "temporal": model.temporal_blocking() and 2 or 1,
        "wrap_axes": "".join(c for i, c in enumerate("xyz") if model.wrap_axes() >> i & 1) or "none",
        "transport": {"inbox": args.inbox,
                      "colo_copy": str(model.domain.transport_options().colo_copy).split(".")[-1].lower(),
                      "completion": args.completion, "fuse_flags": bool(args.fuse_flags)},
    }
    del dd
    del model
    transports = None
    if args.transport_sweep == "on" or (args.transport_sweep == "auto" and world > 1):
        transports = transport_sweep(st, torch, dist, args, world, device, red_dev, axis_cost, objective, topt)

    if rank == 0:
        out = {
            "metric": "Jacobi3D Gcells/s (512^3/GPU weak scaling; halo-exchange GB/s in extra)",
            "value": round(gcells, 3),
            "unit": "Gcells/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (reference Jacobi3D initial condition: 0.5 + hot/cold spheres)",
            "config": {"model": "jacobi3d", "global_batch": cells, "seq_len": max(grid),
                       "grid": list(grid), "grid_rule": args.grid, "partition": args.partition, "per_gpu": args.per_gpu, "radius": 1,
                       "parallelism": f"domain-decomp{n}",
                       **model_cfg,
                       "build": st.build_info()["git_sha"]},
            "extra": {"halo_exchange_GBps": round(xgbs, 3), "halo_exchange_stream_GBps": round(xgbs_stream, 3),
                      "halo_bytes_per_exchange": int(xbytes),
                      "exchange_ms": round(xel / args.exchange_iters * 1e3, 4),
                      "gcells_per_gpu": round(gcells / n, 3), "colo_kernels_us": colo_phases,
                      "transports": transports},
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
