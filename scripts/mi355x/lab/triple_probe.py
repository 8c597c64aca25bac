"""Why a multi-sub-domain temporal=3 model does not take the fused triples: prints the layout facts
stencil7x3_supported checks (wrap axes, radius, alignment, sizes)."""
import stencil2_amd as st

for size, gpus, cost in [((512, 40, 36), [0, 0], (4, 2, 3)), ((512, 20, 64), [0, 0], (4, 3, 2)), ((512, 40, 36), [0], (4, 2, 3))]:
    m = st.AstarothSim(size, gpus=gpus, temporal=3, axis_cost=cost, quantities=2)
    m.init()
    print(size, gpus, "triples", m.temporal_triples(), "pairs", m.temporal_blocking(), "wrap", m.wrap_axes(),
          "overlap", m.overlapping())
    for di in range(m.domain.num_domains()):
        d = m.domain.domain(di)
        r = d.radius()
        print("  dom", di, "size", d.size(), "raw", d.raw_size(), "pitch", d.pitch(0),
              "rad x", r.x(-1), r.x(1), "y", r.y(-1), r.y(1), "z", r.z(-1), r.z(1),
              "curr%16", (d.curr_ptr(0) + 4 * r.x(-1)) % 16, "row_limit", d.row_limit(0), "front_slack", d.front_slack(0))
