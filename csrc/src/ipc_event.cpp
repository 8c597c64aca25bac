// Interprocess event round trip (see stencil/comm/ipc_event.hpp).
#include "stencil/comm/ipc_event.hpp"

#include <hip/hip_runtime_api.h>

#include <chrono>

#include "stencil/comm/tags.hpp"
#include "stencil/kernels/copy.hpp"
#include "stencil/rt/hip_check.hpp"

namespace stencil {

IpcEventReport ipc_event_roundtrip(comm::ProcGroup &pg, int device, double spinS) {
  IpcEventReport rep;
  rep.spinS = spinS;
  const int me = pg.rank(), n = pg.size();
  const uint32_t tagHandle = comm::make_tag(comm::MsgKind::IpcEvent, 0), tagNotify = comm::make_tag(comm::MsgKind::Notify, 0);
  HIP_CHECK(hipSetDevice(device));
  hipStream_t s = nullptr;
  HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev = nullptr;
  int ok = 1;
  if (me == 0) {
    HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventInterprocess));
    hipIpcEventHandle_t h{};
    HIP_CHECK(hipIpcGetEventHandle(&h, ev));
    for (int r = 1; r < n; ++r) pg.send(r, tagHandle, &h, sizeof(h));
  } else {
    hipIpcEventHandle_t h{};
    pg.recv(0, tagHandle, &h, sizeof(h));
    if (hipIpcOpenEventHandle(&ev, h) != hipSuccess) {
      (void)hipGetLastError();
      ok = 0;
      rep.error = "hipIpcOpenEventHandle failed on rank " + std::to_string(me);
    }
  }
  ok = int(pg.allreduce_min_i64(ok));
  if (ok) {
    pg.barrier();
    if (me == 0) {
      spin_device(spinS, s);
      HIP_CHECK(hipEventRecord(ev, s));
      const uint64_t one = 1;
      for (int r = 1; r < n; ++r) pg.send(r, tagNotify, &one, sizeof(one));
      HIP_CHECK(hipStreamSynchronize(s));
      rep.waitedS = spinS;
    } else {
      uint64_t one = 0;
      pg.recv(0, tagNotify, &one, sizeof(one));
      const auto t0 = std::chrono::steady_clock::now();
      HIP_CHECK(hipStreamWaitEvent(s, ev, 0));
      spin_device(0.0, s); // a marker kernel ordered behind the wait
      HIP_CHECK(hipStreamSynchronize(s));
      rep.waitedS = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      // rank 0 enqueued the spin before the notify, so at least most of it is still to run when the wait is enqueued
      if (rep.waitedS < 0.5 * spinS) {
        ok = 0;
        rep.error = "rank " + std::to_string(me) + " did not wait for the recorded work (" +
                    std::to_string(rep.waitedS) + " s of a " + std::to_string(spinS) + " s spin)";
      }
    }
    ok = int(pg.allreduce_min_i64(ok));
  }
  pg.barrier(); // nobody destroys or closes the event while a peer still uses it
  if (ev) (void)hipEventDestroy(ev);
  (void)hipStreamDestroy(s);
  rep.ok = ok != 0;
  return rep;
}

} // namespace stencil
