"""Worker for multi-process tests (launched by conftest.run_ranks). argv[1] = scenario."""
import faulthandler
import os
import sys

import torch

import stencil2_amd as st
from stencil2_amd.ops import jacobi_step_reference
from stencil2_amd.utils.testing import check_exchange, fill_coords


def transport_from_env():
    """TransportOptions of a test scenario (MP_* variables set by the launching test)."""
    t = st.TransportOptions()
    e = os.environ
    t.inbox = getattr(st.TransportOptions.Inbox, e.get("MP_INBOX", "Uncached"))
    t.colo_copy = getattr(st.TransportOptions.Copy, e.get("MP_COLO_COPY", "Store"))
    t.peer_copy = getattr(st.TransportOptions.Copy, e.get("MP_PEER_COPY", "Store"))
    t.completion = getattr(st.TransportOptions.Completion, e.get("MP_COMPLETION", "Kernel"))
    t.jitter_us = int(e.get("MP_JITTER_US", "0"))
    t.fuse_flags = e.get("MP_FUSE_FLAGS", "1") == "1"
    t.fail_ipc_probe = e.get("MP_IPC_PROBE_FAIL") == "1"
    t.fail_rccl_init = e.get("MP_RCCL_INIT_FAIL") == "1"
    t.fail_probe_rank = int(e.get("MP_PROBE_FAIL_RANK", "-1"))
    if e.get("MP_WAIT_TIMEOUT"):
        t.wait_timeout = float(e["MP_WAIT_TIMEOUT"])
    return t


def scenario_exchange(backend, methods, radius_name, size):
    g = st.init_process_group()
    pats = {
        "r1": st.Radius.constant(1),
        "r2": st.Radius.constant(2),
        "fec": st.Radius.face_edge_corner(2, 1, 1),
    }
    r = st.Radius.constant(0)
    r.set_dir(1, 0, 0, 2)
    r.set_dir(-1, 0, 0, 1)
    pats["asym"] = r
    radius = pats[radius_name]
    dd = st.DistributedDomain(*size, group=g)
    dd.set_backend(backend)
    dd.set_transport_options(transport_from_env())
    dd.set_radius(radius)
    if backend == st.Backend.Device:
        dd.set_gpus([0])
    dd.set_methods(methods)
    q = dd.add_data("c", torch.int64)
    q2 = dd.add_data("d", torch.float32)
    dd.realize()
    bad = 0
    for it in range(3):
        fill_coords(dd, q)
        fill_coords(dd, q2)
        print(f"rank {g.rank()} epoch {it} exchange", flush=True)
        dd.exchange()
        bad += check_exchange(dd, q, radius) + check_exchange(dd, q2, radius)
        dd.swap()
    print(f"rank {g.rank()} nodes {g.num_nodes()} bad {bad} plan {[str(e.method) for e in dd.plan()][:3]}")
    return bad


def scenario_canary(backend, methods, radius_name, size, iters=12):
    """Race canary: every iteration writes iteration-tagged interiors, poisons every halo with NaN
    (float) / -1 (int), then exchanges back to back with no barrier between ranks. A halo from another iteration
    (missing credit: reference tx_cuda.cuh:270-283), a surviving poison cell or a touched interior cell fails."""
    g = st.init_process_group()
    radius = {"r1": st.Radius.constant(1), "fec": st.Radius.face_edge_corner(2, 1, 1)}[radius_name]
    dd = st.DistributedDomain(*size, group=g)
    dd.set_backend(backend)
    dd.set_transport_options(transport_from_env())
    dd.set_radius(radius)
    if backend == st.Backend.Device:
        dd.set_gpus([0])
    dd.set_methods(methods)
    q = dd.add_data("c", torch.int64)
    qf = dd.add_data("f", torch.float64)
    dd.realize()
    bad = 0
    for it in range(iters):
        off = it * 10_000_000
        fill_coords(dd, q, offset=off)
        fill_coords(dd, qf, poison=-1, offset=off)
        for di in range(dd.num_domains()):  # NaN-poison the float halos (interior stays)
            t = dd.curr(di, qf)
            inner = dd.curr_interior(di, qf).clone()
            t.fill_(float("nan"))
            dd.curr_interior(di, qf).copy_(inner)
        before = [dd.curr_interior(di, q).clone() for di in range(dd.num_domains())]
        print(f"rank {g.rank()} epoch {it} exchange", flush=True)
        dd.exchange()
        print(f"rank {g.rank()} epoch {it} check", flush=True)
        bad += check_exchange(dd, q, radius, offset=off) + check_exchange(dd, qf, radius, offset=off)
        for di in range(dd.num_domains()):
            bad += int((dd.curr_interior(di, q) != before[di]).sum())
        dd.swap()
    print(f"rank {g.rank()} canary bad {bad}")
    return bad


def scenario_jacobi(backend, methods, size):
    """Jacobi3D (or, with MP_KIND=astaroth, the Astaroth proxy started from an analytic global field) across ranks,
    compared with the torch oracle after 3 single steps and run(5)."""
    g = st.init_process_group()
    gpus = [0] if backend == st.Backend.Device else [0]
    temporal = int(os.environ.get("MP_TEMPORAL", "1"))
    kind = os.environ.get("MP_KIND", "jacobi")
    cost = os.environ.get("MP_AXIS_COST")  # NodeAware cut costs, e.g. "4,2,3" (default: the model's)
    kw = {"axis_cost": tuple(int(v) for v in cost.split(","))} if cost else {}
    if os.environ.get("MP_PARTITION") == "maxlink":  # bench.py's decomposition of the xGMI mesh (1x1xN slabs)
        kw["partition"] = st.PartitionObjective.MaxLink
    if os.environ.get("MP_X_HALO_ALIGN") == "1":
        kw["x_halo_align"] = True
    if kind == "astaroth":
        from stencil2_amd.ops import astaroth_step_reference as ref
        m = st.AstarothSim(size, quantities=1, gpus=gpus, backend=backend, methods=methods, group=g,
                           temporal=temporal, transport=transport_from_env(), **kw)
    else:
        ref = jacobi_step_reference
        m = st.Jacobi3D(size, gpus=gpus, backend=backend, methods=methods, group=g, temporal=temporal,
                        transport=transport_from_env(), **kw)
    m.init()
    L = m.domain.size()
    if kind == "astaroth":
        z = torch.arange(L.z, dtype=torch.float64).view(-1, 1, 1)
        y = torch.arange(L.y, dtype=torch.float64).view(1, -1, 1)
        x = torch.arange(L.x, dtype=torch.float64).view(1, 1, -1)
        u = (torch.sin(0.37 * x + 0.11 * y * y) * torch.cos(0.23 * z + 0.05 * x * y)).to(torch.float32)
        for di in range(m.domain.num_domains()):
            d = m.domain.domain(di)
            o, s = d.origin(), d.size()
            m.interior(di).copy_(u[o.z:o.z + s.z, o.y:o.y + s.y, o.x:o.x + s.x].to(m.interior(di).device))
        if backend == st.Backend.Device:
            torch.cuda.synchronize()
    elif os.environ.get("MP_RANDOM") == "1":  # same random global field on every rank (CPU generator, fixed seed)
        u = torch.rand((L.z, L.y, L.x), generator=torch.Generator().manual_seed(1234))
        for di in range(m.domain.num_domains()):
            d = m.domain.domain(di)
            o, s = d.origin(), d.size()
            m.interior(di).copy_(u[o.z:o.z + s.z, o.y:o.y + s.y, o.x:o.x + s.x].to(m.interior(di).device))
        if backend == st.Backend.Device:
            torch.cuda.synchronize()
    else:
        u = torch.full((L.z, L.y, L.x), 0.5)
    if backend == st.Backend.Device and u.numel() > 1 << 24:  # big grids: the oracle runs on the GPU too
        u = u.cuda()
    if os.environ.get("MP_PREPARE") == "1":
        m.prepare()
    first = int(os.environ.get("MP_SINGLE_STEPS", "3"))
    for _ in range(first):
        m.step()
        u = ref(u)
    pairs = int(os.environ.get("MP_RUN_STEPS", "5"))
    m.run(pairs)  # fused pairs when temporal blocking is on
    for _ in range(pairs):
        u = ref(u)
    bad = 0
    if os.environ.get("MP_TOGGLE_OVERLAP"):  # whole-region pairs, then back to overlapped ones (set_overlap)
        bad += int(not m.can_toggle_overlap())
        if m.can_toggle_overlap():
            modes = ((0, 8), (2, 8), (1, 16), (1, 8))
            if os.environ.get("MP_TOGGLE_MODES"):  # e.g. "2": only that mode, with the default reserve
                modes = tuple((int(c), 8) for c in os.environ["MP_TOGGLE_MODES"])
            k = int(os.environ.get("MP_TOGGLE_STEPS", "4" if len(modes) > 1 else "16"))
            for mode, reserve in modes:
                m.set_overlap_mode(mode)
                m.set_comm_reserve(reserve)
                bad += int(m.overlap_mode() != mode or m.comm_reserve() != reserve)
                m.run(k)
                for _ in range(k):
                    u = ref(u)
    if os.environ.get("MP_EXPECT_TRIPLES") is not None:  # fused triples in the final (whole-region) mode
        bad += int(m.temporal_triples() != (os.environ["MP_EXPECT_TRIPLES"] == "1"))
    m.synchronize()
    for di in range(m.domain.num_domains()):
        d = m.domain.domain(di)
        o, s = d.origin(), d.size()
        got = m.interior(di).to(u.device)
        bad += int((got != u[o.z:o.z + s.z, o.y:o.y + s.y, o.x:o.x + s.x]).sum())
    if os.environ.get("MP_EXPECT_WRAP") is not None:  # axes the fused pairs wrap in-kernel (mask 1=x 2=y 4=z)
        bad += int(m.wrap_axes() != int(os.environ["MP_EXPECT_WRAP"]))
    if os.environ.get("MP_EXPECT_STEP_WRAP") is not None:  # single steps: in-kernel wrap axes, local interior
        bad += int(m.step_wrap_axes() != int(os.environ["MP_EXPECT_STEP_WRAP"]))
        bad += int(not m.local_interior_steps())
    if os.environ.get("MP_EXPECT_OVERLAP") is not None:
        bad += int(m.overlapping() != (os.environ["MP_EXPECT_OVERLAP"] == "1"))
    xb = {k: m.domain.exchange_bytes_for_method(getattr(st.MethodFlags, k))
          for k in ("Staged", "Rccl", "Colocated", "PeerCopy", "Kernel")}
    print(f"rank {g.rank()} jacobi bad {bad} overlap {m.overlapping()} dim {m.domain.placement_dim()} "
          + " ".join(f"bytes_{k}={v}" for k, v in xb.items()))
    return bad


def scenario_selftest(backend, methods, size):
    """realize() with the transport self-test ladder, then the coordinate oracle on the verified transports."""
    g = st.init_process_group()
    r = st.Radius.face_edge_corner(2, 1, 1)
    dd = st.DistributedDomain(*size, group=g)
    dd.set_backend(backend)
    dd.set_transport_options(transport_from_env())
    dd.set_radius(r)
    dd.set_methods(methods)
    dd.set_self_test(True)
    if backend == st.Backend.Device:
        dd.set_gpus([0])
    q = dd.add_data("c", torch.int32)
    dd.realize()
    bad = 0
    for it in range(2):
        fill_coords(dd, q, offset=it)
        dd.exchange()
        bad += check_exchange(dd, q, r, offset=it)
        dd.swap()
    print(f"rank {g.rank()} selftest bad {bad} report [{dd.self_test_report()}] methods "
          f"{st.methods_to_string(dd.methods())}", flush=True)
    return bad


def scenario_localint(backend, methods, size):
    """get_local_interior: shrunk by the stencil reach (2) exactly at the faces whose halo comes from another rank,
    untouched along axes that wrap onto the same rank; always a superset of get_interior()."""
    g = st.init_process_group()
    r = st.Radius.constant(0)
    r.set_face(2)
    r.set_edge(1)
    dd = st.DistributedDomain(*size, group=g)
    dd.set_backend(backend)
    dd.set_radius(r)
    dd.set_methods(methods)
    dd.add_data("d", torch.float32)
    dd.realize()
    bad = 0
    li, full = dd.get_local_interior(2), dd.get_interior()
    dim = dd.placement_dim()
    for di in range(dd.num_domains()):
        d = dd.domain(di)
        o, s = d.origin(), d.size()
        a, b = li[di], full[di]
        for ax, n in (("x", dim.x), ("y", dim.y), ("z", dim.z)):
            lo, hi = getattr(o, ax), getattr(o, ax) + getattr(s, ax)
            want = (lo + 2, hi - 2) if n > 1 else (lo, hi)
            got = (getattr(a.lo, ax), getattr(a.hi, ax))
            bad += got != want
            bad += not (getattr(a.lo, ax) <= getattr(b.lo, ax) and getattr(a.hi, ax) >= getattr(b.hi, ax))
    print(f"rank {g.rank()} dim {dim} localint bad {bad}")
    return bad


def scenario_ipcstress():
    """records / waits of one interprocess event, per receiver-side follow-up mode (lab: where does the HIP
    implementation refuse a wait?)"""
    g = st.init_process_group()
    from stencil2_amd import _C
    for after in (0, 1, 2, 3):
        r = _C.ipc_event_stress(g, 0, int(os.environ.get("MP_ITERS", "100")), after)
        print(f"rank {g.rank()} ipcstress after={after} first_failure={r}", flush=True)
    return 0


def scenario_ipcevent():
    """reference test/test_cuda_mpi_cudaipc.cu:8-45: an interprocess event's handle travels from rank 0 to the other
    ranks and opens there; here the receivers also wait on it behind 0.2 s of rank 0's GPU work"""
    g = st.init_process_group()
    from stencil2_amd import _C
    r = _C.ipc_event_roundtrip(g, 0, 0.2)
    print(f"rank {g.rank()} ipcevent {r}", flush=True)
    return 0 if r["ok"] else 1


def scenario_streamloop(size):
    """blocking exchanges, then stream-ordered exchange_async on a caller (torch) stream, then on the comm streams,
    with the coordinate oracle after each phase (TransportOptions from MP_*)"""
    g = st.init_process_group()
    r = st.Radius.constant(0)
    r.set_face(2)
    dd = st.DistributedDomain(*size, group=g)
    dd.set_transport_options(transport_from_env())
    dd.set_radius(r)
    dd.set_gpus([0])
    dd.set_methods(getattr(st.MethodFlags, "Colocated") | getattr(st.MethodFlags, "Kernel"))
    q = dd.add_data("c", torch.int64)
    dd.realize()
    bad = 0
    xs = torch.cuda.Stream()
    iters = int(os.environ.get("MP_ITERS", "4"))
    for phase in ("blocking", "caller", "comm"):
        for it in range(iters):
            fill_coords(dd, q, offset=it)
            if phase == "blocking":
                dd.exchange()
            else:
                dd.exchange_async(xs.cuda_stream if phase == "caller" else 0, 0)
                xs.synchronize()
                dd.sync_exchange()
            bad += check_exchange(dd, q, r, offset=it)
            dd.swap()
        print(f"rank {g.rank()} phase {phase} bad {bad}", flush=True)
    import time
    n = max(6, 2 * iters)
    t0 = time.perf_counter()
    for it in range(n):  # back to back on the caller stream, one synchronize
        dd.exchange_async(xs.cuda_stream, 0)
        dd.swap()
    xs.synchronize()
    dd.sync_exchange()
    dt = (time.perf_counter() - t0) / n * 1e6
    fill_coords(dd, q, offset=99)
    dd.exchange()
    bad += check_exchange(dd, q, r, offset=99)
    if os.environ.get("MP_SWITCH") == "1":  # completion switched between exchanges (every rank at the same point)
        C = st.TransportOptions.Completion
        for k, c in enumerate((C.Kernel, C.IpcEvent, C.StreamOp, C.IpcEvent, C.Kernel)):
            dd.set_completion(c)
            for it in range(30 if c == C.IpcEvent else 3):
                fill_coords(dd, q, offset=1000 * k + it)
                dd.exchange()
                bad += check_exchange(dd, q, r, offset=1000 * k + it)
                dd.swap()
        print(f"rank {g.rank()} switch bad {bad}", flush=True)
    print(f"rank {g.rank()} streamloop bad {bad} back-to-back {dt:.1f} us per exchange", flush=True)
    return bad


def scenario_ipcseq(size):
    """two Completion::IpcEvent domains built one after the other on ONE process group (same channel tags:
    the first one's undrained Acks would reach the second), and in the second one more than 40 stream-ordered
    exchanges enqueued behind a long spin of the comm stream, so the host runs far ahead of the device while the
    sender replaces its event (every 24 records) -- replaced events must outlive the queued records / waits."""
    g = st.init_process_group()
    r = st.Radius.constant(0)
    r.set_face(2)
    bad = 0
    from stencil2_amd import _C
    for k in range(2):
        t = transport_from_env()
        t.completion = st.TransportOptions.Completion.IpcEvent
        dd = st.DistributedDomain(*size, group=g)
        dd.set_transport_options(t)
        dd.set_radius(r)
        dd.set_gpus([0])
        dd.set_methods(st.MethodFlags.Colocated | st.MethodFlags.Kernel)
        q = dd.add_data("c", torch.int64)
        dd.realize()
        for it in range(3):
            fill_coords(dd, q, offset=100 * k + it)
            dd.exchange()
            bad += check_exchange(dd, q, r, offset=100 * k + it)
            dd.swap()
        if k == 1:
            fill_coords(dd, q, offset=7)
            _C.spin_device(1.0, dd.comm_stream(0))
            n = int(os.environ.get("MP_ITERS", "48"))
            for it in range(n):  # an even number: the field is back in the buffer fill_coords wrote
                dd.exchange_async(0, 0)
                dd.swap()
            dd.sync_exchange()
            bad += check_exchange(dd, q, r, offset=7)
        print(f"rank {g.rank()} ipcseq domain {k} bad {bad}", flush=True)
        del dd
    print(f"rank {g.rank()} ipcseq bad {bad}", flush=True)
    return bad


def main():
    # a stalled rank dumps every thread's Python stack (its C++ frames show as the native call it is in) so a hang
    # names its rank, scenario and phase; repeated, in case the first dump lands before the stall
    faulthandler.enable()
    faulthandler.dump_traceback_later(float(os.environ.get("MP_STALL_DUMP_S", "40")), repeat=True)
    sc = sys.argv[1]
    backend = st.Backend.Device if os.environ.get("MP_DEVICE") == "1" else st.Backend.Host
    methods = st.MethodFlags.None_
    for name in os.environ.get("MP_METHODS", "All").split("|"):
        methods = methods | getattr(st.MethodFlags, name)
    if sc == "exchange":
        bad = scenario_exchange(backend, methods, sys.argv[2], tuple(int(v) for v in sys.argv[3].split(",")))
    elif sc == "canary":
        bad = scenario_canary(backend, methods, sys.argv[2], tuple(int(v) for v in sys.argv[3].split(",")))
    elif sc == "selftest":
        bad = scenario_selftest(backend, methods, tuple(int(v) for v in sys.argv[2].split(",")))
    elif sc == "localint":
        bad = scenario_localint(backend, methods, tuple(int(v) for v in sys.argv[2].split(",")))
    elif sc == "streamloop":
        bad = scenario_streamloop(tuple(int(v) for v in sys.argv[2].split(",")))
    elif sc == "ipcstress":
        bad = scenario_ipcstress()
    elif sc == "ipcseq":
        bad = scenario_ipcseq(tuple(int(v) for v in sys.argv[2].split(",")))
    elif sc == "ipcevent":
        bad = scenario_ipcevent()
    elif sc == "jacobi":
        bad = scenario_jacobi(backend, methods, tuple(int(v) for v in sys.argv[2].split(",")))
    else:
        raise SystemExit("unknown scenario")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
