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

std::string ipc_event_stress(comm::ProcGroup &pg, int device, int n, int after) {
  const int me = pg.rank();
  const uint32_t tagHandle = comm::make_tag(comm::MsgKind::IpcEvent, 1), tagNotify = comm::make_tag(comm::MsgKind::Notify, 1),
                 tagAck = comm::make_tag(comm::MsgKind::Ack, 1);
  HIP_CHECK(hipSetDevice(device));
  hipStream_t s = nullptr;
  HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev = nullptr;
  int failedAt = -1;
  std::string err;
  auto note = [&](int it, hipError_t e, const char *what) {
    if (e == hipSuccess || failedAt >= 0) return;
    (void)hipGetLastError();
    failedAt = it;
    err = std::string(what) + ": " + hipGetErrorString(e);
  };
  if (me == 0) {
    HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming | hipEventInterprocess));
    hipIpcEventHandle_t h{};
    HIP_CHECK(hipIpcGetEventHandle(&h, ev));
    if (pg.size() > 1) pg.send(1, tagHandle, &h, sizeof(h));
  } else if (me == 1) {
    hipIpcEventHandle_t h{};
    pg.recv(0, tagHandle, &h, sizeof(h));
    note(-1, hipIpcOpenEventHandle(&ev, h), "hipIpcOpenEventHandle");
  }
  for (int it = 0; it < n && me <= 1 && pg.size() > 1; ++it) {
    int64_t st = failedAt;
    if (me == 0) {
      spin_device(20e-6, s);
      note(it, hipEventRecord(ev, s), "hipEventRecord");
      st = failedAt;
      pg.send(1, tagNotify, &st, sizeof(st));
      pg.recv(1, tagAck, &st, sizeof(st));
      if (st >= 0 && failedAt < 0) failedAt = int(st), err = "peer";
    } else {
      pg.recv(0, tagNotify, &st, sizeof(st));
      if (after == 3) {
        note(it, hipEventSynchronize(ev), "hipEventSynchronize");
      } else {
        note(it, hipStreamWaitEvent(s, ev, 0), "hipStreamWaitEvent");
        spin_device(0.0, s);
        if (after >= 1) note(it, hipStreamSynchronize(s), "hipStreamSynchronize");
        if (after >= 2) {
          const hipError_t q = hipEventQuery(ev);
          if (q != hipErrorNotReady) note(it, q, "hipEventQuery");
          else (void)hipGetLastError();
        }
      }
      st = failedAt;
      pg.send(0, tagAck, &st, sizeof(st));
    }
    if (failedAt >= 0) break;
  }
  (void)hipStreamSynchronize(s);
  pg.barrier();
  if (ev) (void)hipEventDestroy(ev);
  (void)hipStreamDestroy(s);
  return std::to_string(failedAt) + ":" + err;
}

} // namespace stencil
