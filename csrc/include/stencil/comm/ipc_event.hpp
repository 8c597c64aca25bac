#pragma once
// Interprocess HIP events between co-located ranks: the primitive of TransportOptions::Completion::IpcEvent.
// Parity: reference test/test_cuda_mpi_cudaipc.cu:8-45 (create an interprocess event on rank 0, send its handle, open
// it on rank 1) and tx_cuda.cuh:231-240 / :366-372 (record after the copy, cudaStreamWaitEvent before the unpack).
#include <string>

#include "stencil/comm/proc_group.hpp"

namespace stencil {

struct IpcEventReport {
  bool ok = false;
  double spinS = 0;   // how long rank 0's GPU was kept busy before it recorded the event
  double waitedS = 0; // receivers: host time from the notify until their stream (waiting on the event) drained
  std::string error;
};

// Collective over every rank of `pg` (all on one node): rank 0 creates an interprocess event (hipEventDisableTiming |
// hipEventInterprocess), sends its handle to every other rank, which opens it (hipIpcOpenEventHandle). Rank 0 then
// keeps its GPU busy for `spinS` seconds, records the event behind that work and notifies the others at once; each
// receiver orders a marker on its stream after hipStreamWaitEvent on the opened event and measures how long the
// stream takes to drain. ok: every handle opened and every receiver's wait covered (most of) the spin.
IpcEventReport ipc_event_roundtrip(comm::ProcGroup &pg, int device, double spinS);

// Repeated records of one interprocess event (rank 0) and waits on it (rank 1), `n` times, each wait followed on
// the receiver by `after`: 0 nothing, 1 hipStreamSynchronize of the waiting stream, 2 that plus hipEventQuery on
// the opened event, 3 hipEventSynchronize on the opened event instead of the stream wait. Returns the first
// iteration whose HIP call failed (-1: none) and that call's error string, as "iteration:error".
std::string ipc_event_stress(comm::ProcGroup &pg, int device, int n, int after);

} // namespace stencil
