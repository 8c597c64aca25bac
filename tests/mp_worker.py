"""Worker for multi-process tests (launched by conftest.run_ranks). argv[1] = scenario."""
import os
import sys

import torch

import stencil2_amd as st
from stencil2_amd.ops import jacobi_step_reference
from stencil2_amd.utils.testing import check_exchange, fill_coords


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
        dd.exchange()
        bad += check_exchange(dd, q, radius) + check_exchange(dd, q2, radius)
        dd.swap()
    print(f"rank {g.rank()} nodes {g.num_nodes()} bad {bad} plan {[str(e.method) for e in dd.plan()][:3]}")
    return bad


def scenario_jacobi(backend, methods, size):
    g = st.init_process_group()
    gpus = [0] if backend == st.Backend.Device else [0]
    m = st.Jacobi3D(size, gpus=gpus, backend=backend, methods=methods, group=g)
    m.init()
    L = m.domain.size()
    u = torch.full((L.z, L.y, L.x), 0.5)
    for _ in range(3):
        m.step()
        u = jacobi_step_reference(u)
    m.synchronize()
    bad = 0
    for di in range(m.domain.num_domains()):
        d = m.domain.domain(di)
        o, s = d.origin(), d.size()
        got = m.interior(di).cpu()
        bad += int((got != u[o.z:o.z + s.z, o.y:o.y + s.y, o.x:o.x + s.x]).sum())
    print(f"rank {g.rank()} jacobi bad {bad}")
    return bad


def main():
    sc = sys.argv[1]
    backend = st.Backend.Device if os.environ.get("MP_DEVICE") == "1" else st.Backend.Host
    methods = st.MethodFlags.None_
    for name in os.environ.get("MP_METHODS", "All").split("|"):
        methods = methods | getattr(st.MethodFlags, name)
    if sc == "exchange":
        bad = scenario_exchange(backend, methods, sys.argv[2], tuple(int(v) for v in sys.argv[3].split(",")))
    elif sc == "jacobi":
        bad = scenario_jacobi(backend, methods, tuple(int(v) for v in sys.argv[2].split(",")))
    else:
        raise SystemExit("unknown scenario")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
