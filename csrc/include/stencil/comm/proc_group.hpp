#pragma once
// Host-side process group: bootstrap, control plane and the host-staged data plane.
//
// The reference relies on MPI for all of this (MPI_Comm_split_type, Allgather, Bcast, Isend/Irecv;
// reference include/stencil/mpi_topology.hpp:18-36, src/stencil.cu:358-361, tx_cuda.cuh:638-649).
// Here it is a small native TCP full mesh so the runtime has no MPI dependency and the same binary runs
// under `torchrun` (RANK/WORLD_SIZE/MASTER_ADDR), a plain launcher, or as a single process.
// GPU data never goes through this layer except on the host-staged fallback transport; GPU-resident
// traffic uses HIP IPC (xGMI) or RCCL.
#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace stencil {
namespace comm {

class ProcGroup {
public:
  virtual ~ProcGroup() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;

  // node name of rank r (gethostname(), or STENCIL_HOSTNAME to fake multi-node layouts in tests)
  virtual const std::string &hostname(int r) const = 0;

  // tagged point-to-point. Tags with the top bit set are reserved for collectives.
  // send() never blocks on the receiver posting a recv (a reader thread drains every socket).
  virtual void send(int dst, uint32_t tag, const void *buf, size_t n) = 0;
  virtual void recv(int src, uint32_t tag, void *buf, size_t n) = 0;
  // non-blocking probe-and-receive: returns true and fills buf if a matching message is queued
  virtual bool try_recv(int src, uint32_t tag, void *buf, size_t n) = 0;

  // collectives (every rank must call them in the same order)
  virtual void barrier() = 0;
  // barrier that gives up after timeout_s (returns false; the group's collective sequence is then out of step, so
  // only use it on the way out, e.g. in a destructor)
  virtual bool barrier_for(double timeout_s) {
    (void)timeout_s;
    barrier();
    return true;
  }
  // receive timeout of blocking recv / collectives (seconds)
  virtual void set_timeout(double timeout_s) { (void)timeout_s; }
  virtual double timeout() const { return 0; }
  // collective: a new group over the same ranks with its own connections, mailboxes and collective sequence, whose
  // blocking receives give up after timeout_s. Work that may fail on some ranks only (the transport self-test probe)
  // runs on a fork: when one rank abandons it mid-sequence, the others time out there and this group's own
  // collective sequence stays in step. A size-1 group returns itself.
  virtual std::shared_ptr<ProcGroup> fork(double timeout_s) = 0;
  virtual void bcast(void *buf, size_t n, int root) = 0;
  virtual void allgather(const void *in, size_t n, void *out) = 0;                           // out: size()*n bytes
  virtual void gatherv(const void *in, size_t n, std::vector<std::vector<char>> *out, int root) = 0; // root only
  double allreduce_max(double v);
  double allreduce_sum(double v);
  uint64_t allreduce_sum_u64(uint64_t v);
  int64_t allreduce_min_i64(int64_t v);

  // ranks on the same node as this rank (sorted), and this rank's index among them
  std::vector<int> colocated_ranks() const;
  int colocated_rank() const;
  int colocated_size() const { return int(colocated_ranks().size()); }
  bool colocated(int r) const { return hostname(r) == hostname(rank()); }
  int num_nodes() const;
};

// single process, size 1
std::shared_ptr<ProcGroup> make_single_group();

// TCP full mesh. Rank 0 listens on master_addr:master_port for the rendezvous.
std::shared_ptr<ProcGroup> make_tcp_group(int rank, int size, const std::string &master_addr, int master_port,
                                          double timeout_s = 600.0);

// From the environment: STENCIL_RANK/RANK, STENCIL_WORLD_SIZE/WORLD_SIZE,
// STENCIL_MASTER_ADDR/MASTER_ADDR, STENCIL_MASTER_PORT or MASTER_PORT+1. size==1 -> single group.
std::shared_ptr<ProcGroup> make_group_from_env();

// process-wide default group used by DistributedDomain when none is given
std::shared_ptr<ProcGroup> default_group();
void set_default_group(std::shared_ptr<ProcGroup> g);

// an unused TCP port on this host (for the rank-0 rendezvous)
int find_free_port();

} // namespace comm
} // namespace stencil
