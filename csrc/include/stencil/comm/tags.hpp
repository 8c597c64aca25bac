#pragma once
// Message tags of the host control/data plane (the native process group).
// Parity: reference include/stencil/tx_common.hpp:23-110 (MsgKind {ColocatedEvt, Mem, Dev, Notify, Other} and
// make_tag packing kind | dir | payload into 24 bits). The reference's remote path uses a separate
// `(src&0xF)<<4 | dst&0xF` scheme on the same communicator, so tags of different kinds can collide and more than
// 8 sub-domains per rank trip an assert. Here every tag is built by make_tag: 3 kind bits and a
// 28-bit (src sub-domain, dst sub-domain) pair key, checked for overflow; the top bit stays reserved for the
// process group's collectives. RCCL itself has no tags: its matching order is the canonical channel order.
#include <cstdint>

#include "stencil/rt/logging.hpp"

namespace stencil {
namespace comm {

enum class MsgKind : uint32_t {
  Data = 0,      // host-staged halo payload of one (src, dst) channel
  IpcInbox = 1,  // HIP IPC handle of a receiver's inbox block
  IpcCredit = 2, // HIP IPC handle of a sender's credit block
  Probe = 3,     // pre-flight IPC probe
  Ctrl = 4,      // anything else (checkpoint/metadata)
  IpcEvent = 5,  // HIP IPC handle of a sender's interprocess event (Completion::IpcEvent)
  Notify = 6,    // "recorded epoch e" from a sender (reference MsgKind::Notify, tx_common.hpp)
  Ack = 7,       // "waited on epoch e" from a receiver (keeps a sender from re-recording an event too early)
};

constexpr int kTagPairBits = 28;
constexpr uint32_t kTagPairMask = (1u << kTagPairBits) - 1;
constexpr int64_t kTagMaxSubdomains = int64_t(1) << (kTagPairBits / 2); // every pair key fits
constexpr uint32_t kTagReserved = 0x80000000u; // collectives of the process group

// pair key of the channel src sub-domain -> dst sub-domain among numSub sub-domains (linear indices)
inline uint32_t make_tag(MsgKind kind, int64_t srcLinear, int64_t dstLinear, int64_t numSub) {
  STENCIL_REQUIRE(srcLinear >= 0 && dstLinear >= 0 && srcLinear < numSub && dstLinear < numSub,
                  "tag endpoints out of range");
  STENCIL_REQUIRE(numSub <= kTagMaxSubdomains, "too many sub-domains for the tag space: " << numSub);
  const int64_t key = srcLinear * numSub + dstLinear;
  return (uint32_t(kind) << kTagPairBits) | uint32_t(key);
}
// a tag with a plain payload (e.g. a rank)
inline uint32_t make_tag(MsgKind kind, uint32_t payload) {
  STENCIL_REQUIRE(payload <= kTagPairMask, "tag payload overflow");
  return (uint32_t(kind) << kTagPairBits) | payload;
}
inline MsgKind tag_kind(uint32_t tag) { return MsgKind((tag >> kTagPairBits) & 0x7u); }
inline uint32_t tag_payload(uint32_t tag) { return tag & kTagPairMask; }

} // namespace comm
} // namespace stencil
