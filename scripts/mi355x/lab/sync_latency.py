"""Host-side latency of run(n) + synchronize(): hipGraph replay (run(20) as one prepared graph) vs eager launches, on
the 512^3 triple model and on a tiny model (the launch + wake-up floor, ~41-44 us on MI355X; a polling synchronize
measured the same as hipStreamSynchronize, profiles/r6/r6ag). Median us of 10 runs per round, rounds interleaved.
python scripts/mi355x/lab/sync_latency.py"""
import json
import os
import sys
import time

sys.path.append(os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))))
import stencil2_amd as st  # noqa: E402

for shape, n, graph in (((512, 512, 512), 20, True), ((512, 512, 512), 20, False), ((64, 64, 64), 1, True),
                        ((64, 64, 64), 1, False), ((64, 64, 64), 3, False)):
    m = st.Jacobi3D(shape, gpus=[0], temporal=3, use_graph=graph)
    m.init()
    m.prepare([n])
    m.run(5 * n)
    m.synchronize()
    res = []
    for rnd in range(4):
        ts = []
        for _ in range(10):
            t0 = time.perf_counter()
            m.run(n)
            m.synchronize()
            ts.append(time.perf_counter() - t0)
        res.append(round(sorted(ts)[len(ts) // 2] * 1e6, 1))
    print(json.dumps({"shape": shape, "steps": n, "graph": graph, "median_us": res}), flush=True)
    del m
