#pragma once
// Message packing: aggregate every halo message from one sub-domain to one neighbour into one buffer.
// Parity: reference include/stencil/packer.cuh (Packer/Unpacker interfaces :22-48, DevicePacker :71-192,
// DeviceUnpacker :252-364): messages sorted by direction, each quantity aligned to its element size, sending along
// `dir` packs the interior slab on the dir side with the extent of the receiver's -dir halo. Instead of one kernel
// launch per message captured into a CUDA graph, a prepared Packer owns one descriptor copy plan per buffer parity
// (curr/next swap) and packs everything with a single launch.
#include <memory>
#include <vector>

#include "stencil/domain/local_domain.hpp"
#include "stencil/kernels/copy.hpp"

namespace stencil {

// one halo message: sent along `dir` from sub-domain srcId (on the sending rank) to dstId (on the receiving rank)
struct Message {
  Dim3 dir;
  int srcId, dstId;
  bool operator<(const Message &o) const { return dir < o.dir; }
  bool operator==(const Message &o) const { return dir == o.dir && srcId == o.srcId && dstId == o.dstId; }
};

int64_t packed_size(const LocalDomain &dom, const std::vector<Message> &sortedMsgs);
// segments: interior slabs -> dense buffer (pack) / dense buffer -> -dir halos (unpack); `curr` picks the physical
// buffer that is "curr" in this variant
void build_pack_segs(const LocalDomain &dom, const std::vector<Message> &sortedMsgs, char *buf, bool curr,
                     std::vector<CopySeg> &out);
void build_unpack_segs(const LocalDomain &dom, const std::vector<Message> &sortedMsgs, char *buf, bool curr,
                       std::vector<CopySeg> &out);
// direct same-process translate: src interior slab -> dst -dir halo. xSectors: copy x faces as whole 64-B sectors
// where both layouts allow it (the extra cells land in the receiver's row padding), see build_translate_segs_q
void build_translate_segs(const LocalDomain &src, const LocalDomain &dst, const Dim3 &dir, bool curr,
                          std::vector<CopySeg> &out, bool xSectors = false);
// same for one quantity
void build_translate_segs_q(const LocalDomain &src, const LocalDomain &dst, const Dim3 &dir, bool curr, int64_t q,
                            std::vector<CopySeg> &out, bool xSectors = false);

class PackerBase {
public:
  explicit PackerBase(hipStream_t stream = nullptr) : stream_(stream) {}
  virtual ~PackerBase();
  PackerBase(const PackerBase &) = delete;
  PackerBase &operator=(const PackerBase &) = delete;
  int64_t size() const { return size_; }
  void *data() const { return buf_; }
  void set_stream(hipStream_t s) { stream_ = s; }

protected:
  void prepare_impl(LocalDomain *dom, std::vector<Message> msgs, bool pack);
  void run();
  LocalDomain *dom_ = nullptr;
  std::vector<Message> msgs_;
  int64_t size_ = 0;
  char *buf_ = nullptr;
  bool device_ = false;
  hipStream_t stream_;
  std::vector<CopySeg> segs_[2];
  CopyPlan plan_[2];
};

class Packer : public PackerBase {
public:
  using PackerBase::PackerBase;
  void prepare(LocalDomain *dom, const std::vector<Message> &msgs) { prepare_impl(dom, msgs, true); }
  void pack() { run(); }
};

class Unpacker : public PackerBase {
public:
  using PackerBase::PackerBase;
  void prepare(LocalDomain *dom, const std::vector<Message> &msgs) { prepare_impl(dom, msgs, false); }
  void unpack() { run(); }
};

} // namespace stencil
