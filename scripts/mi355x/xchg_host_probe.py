import json, time, torch, stencil2_amd as st
m = st.Jacobi3D((512, 512, 512), gpus=[0], temporal=2); m.init(); m.run(2); m.synchronize()
dd = m.domain; dd.set_comm_max_blocks(0); N = 50
s = torch.cuda.Stream(); h = s.cuda_stream
o = {}
def tm(k, f):
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(N): f()
    o[k + "_host"] = (time.perf_counter() - t) / N * 1e6
    torch.cuda.synchronize(); o[k] = (time.perf_counter() - t) / N * 1e6
tm("swap", lambda: dd.swap())
tm("attr", lambda: s.cuda_stream)
tm("async_side", lambda: dd.exchange_async(h, 0))
tm("async_own", lambda: dd.exchange_async(0, 0))
tm("async_side2", lambda: dd.exchange_async(h, 0))
print(json.dumps({k: round(v, 1) for k, v in o.items()}), flush=True)
