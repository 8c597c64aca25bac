#include "stencil/domain/local_domain.hpp"

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "stencil/rt/hip_check.hpp"
#include "stencil/rt/trace.hpp"

namespace stencil {

LocalDomain::LocalDomain(const Dim3 &sz, const Dim3 &origin, int dev, Backend backend)
    : sz_(sz), origin_(origin), dev_(dev), backend_(backend) {}

LocalDomain::LocalDomain(LocalDomain &&o) noexcept
    : sz_(o.sz_), origin_(o.origin_), radius_(o.radius_), dev_(o.dev_), backend_(o.backend_), pad_(o.pad_),
      xHaloAlign_(o.xHaloAlign_), sharedLine_(o.sharedLine_), sharedActive_(o.sharedActive_), interiorAlign_(o.interiorAlign_), rowPadLines_(o.rowPadLines_), guard_(o.guard_), realized_(o.realized_), parity_(o.parity_), elemSize_(std::move(o.elemSize_)), dtype_(std::move(o.dtype_)),
      names_(std::move(o.names_)), pitchX_(std::move(o.pitchX_)), padX_(std::move(o.padX_)), tailX_(std::move(o.tailX_)),
      curr_(std::move(o.curr_)), next_(std::move(o.next_)) {
  base_[0] = std::move(o.base_[0]);
  base_[1] = std::move(o.base_[1]);
  o.base_[0].clear();
  o.base_[1].clear();
  o.realized_ = false;
}

LocalDomain::~LocalDomain() { free_all(); }

void LocalDomain::free_all() {
  for (int b = 0; b < 2; ++b) {
    for (void *p : base_[b]) {
      if (!p) continue;
      if (backend_ == Backend::Device) {
        set_device();
        (void)hipFree(p);
      } else {
        std::free(p);
      }
    }
    base_[b].clear();
  }
  curr_.clear();
  next_.clear();
}

void LocalDomain::set_device() const {
  if (backend_ == Backend::Device) HIP_CHECK(hipSetDevice(dev_));
}

int64_t LocalDomain::add_data(int64_t elemSize, const std::string &name, DType dtype) {
  STENCIL_REQUIRE(!realized_, "add_data after realize");
  STENCIL_REQUIRE(elemSize > 0, "element size must be positive");
  elemSize_.push_back(elemSize);
  dtype_.push_back(dtype);
  names_.push_back(name);
  return int64_t(elemSize_.size()) - 1;
}

int64_t LocalDomain::buffer_bytes(int64_t qi) const {
  const Dim3 p = pitch(qi);
  return p.x * p.y * p.z * elem_size(qi);
}

// x halos of at most this many bytes go into the interior's first / last 64-B sector (set_x_halo_align)
static constexpr int64_t kMaxAlignedHaloBytes = 48;

void LocalDomain::realize() {
  STENCIL_REQUIRE(!realized_, "LocalDomain realized twice");
  TraceRange tr("LocalDomain::realize");
  const Dim3 raw = raw_size();
  const int64_t nq = num_data();
  pitchX_.assign(size_t(nq), raw.x);
  padX_.assign(size_t(nq), 0);
  tailX_.assign(size_t(nq), 0);
  int64_t total = 0;
  const int64_t rxm = radius_.x(-1), rxp = radius_.x(1);
  const bool haloAligned = xHaloAlign_ && pad_;
  guard_ = haloAligned ? 128 : 0;
  // shared halo lines: every quantity's interior on an alignment unit and both x halos within one unit
  sharedActive_ = sharedLine_ && pad_ && !haloAligned;
  for (int64_t q = 0; q < nq && sharedActive_; ++q) {
    const int64_t es = elemSize_[q];
    sharedActive_ = interiorAlign_ % es == 0 && (rxm + rxp) * es <= interiorAlign_ && (128 % es == 0);
  }
  for (int64_t q = 0; q < nq; ++q) {
    const int64_t es = elemSize_[q];
    if (sharedActive_) {
      const int64_t perLine = interiorAlign_ / es, rowAlign = 128 / es;
      padX_[q] = (perLine - (rxm % perLine)) % perLine;
      // row r's raw end (padX + raw.x) stays within row r+1's front padding: raw.x <= pitch; the interior start
      // (padX + rxm) is on a unit in every row since the pitch is a multiple of the unit
      pitchX_[q] = round_up(std::max(raw.x, int64_t(1)), std::max(perLine, rowAlign));
      const int64_t tail = (16 % es == 0) ? 16 / es + 1 : 1;
      tailX_[q] = padX_[q] + tail + rowAlign; // the last row's halo + vector over-reads stay allocated
      total += 2 * (buffer_bytes(q) + tailX_[q] * es);
      continue;
    }
    if (pad_ && interiorAlign_ % es == 0) {
      const int64_t perLine = interiorAlign_ / es; // elements per interior alignment unit (64 or 128 B)
      if (haloAligned && 16 % es == 0 && rxm * es <= kMaxAlignedHaloBytes && rxp * es <= kMaxAlignedHaloBytes) {
        // interior at the first 16-B boundary at or after the -x halo (inside the row's first sector)
        padX_[q] = (round_up(rxm * es, 16) - rxm * es) / es;
      } else {
        padX_[q] = (perLine - (rxm % perLine)) % perLine;
      }
      const int64_t rowAlign = (128 % es == 0) ? 128 / es : 1;
      // tail: one 16-B vector + 1 element so vectorized row sweeps never leave the allocation
      const int64_t tail = (16 % es == 0) ? 16 / es + 1 : 1;
      pitchX_[q] = round_up(padX_[q] + raw.x + tail, rowAlign) + int64_t(rowPadLines_) * rowAlign;
    }
    total += 2 * (buffer_bytes(q) + guard_);
  }
  if (backend_ == Backend::Device) {
    set_device();
    size_t freeB = 0, totalB = 0;
    if (hipMemGetInfo(&freeB, &totalB) == hipSuccess) {
      STENCIL_REQUIRE(uint64_t(total) <= uint64_t(freeB),
                      "LocalDomain needs " << total << " B of HBM but only " << freeB << " B of " << totalB
                                           << " B are free on device " << dev_);
    }
  }
  for (int b = 0; b < 2; ++b) base_[b].assign(size_t(nq), nullptr);
  curr_.assign(size_t(nq), nullptr);
  next_.assign(size_t(nq), nullptr);
  for (int64_t q = 0; q < nq; ++q) {
    const int64_t bytes = buffer_bytes(q) + guard_ + tailX_[q] * elemSize_[q];
    for (int b = 0; b < 2; ++b) {
      void *p = nullptr;
      if (backend_ == Backend::Device) {
        HIP_CHECK(hipMalloc(&p, size_t(bytes)));
        HIP_CHECK(hipMemset(p, 0, size_t(bytes)));
      } else {
        p = std::aligned_alloc(256, size_t(round_up(bytes, 256)));
        STENCIL_REQUIRE(p, "host allocation of " << bytes << " B failed");
        std::memset(p, 0, size_t(bytes));
      }
      base_[b][q] = p;
    }
    // raw [0,0,0] sits padX elements into the first row (which starts guard_ bytes into the allocation)
    curr_[q] = static_cast<char *>(base_[0][q]) + guard_ + padX_[q] * elemSize_[q];
    next_[q] = static_cast<char *>(base_[1][q]) + guard_ + padX_[q] * elemSize_[q];
  }
  realized_ = true;
}

Dim3 LocalDomain::halo_pos(const Dim3 &dir, bool halo) const {
  Dim3 r;
  const int64_t rx = radius_.x(-1), ry = radius_.y(-1), rz = radius_.z(-1);
  r.x = dir.x == 1 ? sz_.x + (halo ? rx : 0) : (dir.x == -1 ? (halo ? 0 : rx) : rx);
  r.y = dir.y == 1 ? sz_.y + (halo ? ry : 0) : (dir.y == -1 ? (halo ? 0 : ry) : ry);
  r.z = dir.z == 1 ? sz_.z + (halo ? rz : 0) : (dir.z == -1 ? (halo ? 0 : rz) : rz);
  return r;
}

Rect3 LocalDomain::halo_coords(const Dim3 &dir, bool halo) const {
  Dim3 pos = halo_pos(dir, halo) - Dim3(radius_.x(-1), radius_.y(-1), radius_.z(-1)) + origin_;
  return Rect3(pos, pos + halo_extent(dir));
}

StridedBox LocalDomain::box(int64_t qi, bool curr, const Dim3 &pos) const {
  const Dim3 p = pitch(qi);
  const int64_t es = elem_size(qi);
  StridedBox b;
  b.ystride = p.x * es;
  b.zstride = p.x * p.y * es;
  char *base = static_cast<char *>(curr ? curr_data(qi) : next_data(qi));
  b.base = base + pos.x * es + pos.y * b.ystride + pos.z * b.zstride;
  return b;
}

void LocalDomain::swap() {
  std::swap(curr_, next_);
  parity_ ^= 1;
}

std::vector<unsigned char> LocalDomain::region_to_host(const Dim3 &pos, const Dim3 &ext, int64_t qi, bool curr) const {
  STENCIL_REQUIRE(realized_, "region_to_host before realize");
  const int64_t es = elem_size(qi);
  std::vector<unsigned char> out(size_t(ext.flatten() * es));
  if (out.empty()) return out;
  StridedBox dense;
  dense.ystride = ext.x * es;
  dense.zstride = ext.x * ext.y * es;
  if (backend_ == Backend::Host) {
    dense.base = reinterpret_cast<char *>(out.data());
    std::vector<CopySeg> segs{make_copy_seg(box(qi, curr, pos), dense, ext, es)};
    finalize_segs(segs);
    copy_segs_host(segs);
    return out;
  }
  set_device();
  char *dbuf = nullptr;
  HIP_CHECK(hipMalloc(&dbuf, out.size()));
  dense.base = dbuf;
  copy_segs_device_sync({make_copy_seg(box(qi, curr, pos), dense, ext, es)}, dev_);
  HIP_CHECK(hipMemcpy(out.data(), dbuf, out.size(), hipMemcpyDeviceToHost));
  HIP_CHECK(hipFree(dbuf));
  return out;
}

void LocalDomain::region_from_host(const Dim3 &pos, const Dim3 &ext, int64_t qi, const void *src, bool curr) {
  STENCIL_REQUIRE(realized_, "region_from_host before realize");
  const int64_t es = elem_size(qi);
  const size_t bytes = size_t(ext.flatten() * es);
  if (!bytes) return;
  StridedBox dense;
  dense.ystride = ext.x * es;
  dense.zstride = ext.x * ext.y * es;
  if (backend_ == Backend::Host) {
    dense.base = const_cast<char *>(static_cast<const char *>(src));
    std::vector<CopySeg> segs{make_copy_seg(dense, box(qi, curr, pos), ext, es)};
    finalize_segs(segs);
    copy_segs_host(segs);
    return;
  }
  set_device();
  char *dbuf = nullptr;
  HIP_CHECK(hipMalloc(&dbuf, bytes));
  HIP_CHECK(hipMemcpy(dbuf, src, bytes, hipMemcpyHostToDevice));
  dense.base = dbuf;
  copy_segs_device_sync({make_copy_seg(dense, box(qi, curr, pos), ext, es)}, dev_);
  HIP_CHECK(hipFree(dbuf));
}

void LocalDomain::fill_bytes(int64_t qi, uint8_t v, bool curr, bool next) {
  const int64_t bytes = buffer_bytes(qi) + tailX_.at(size_t(qi)) * elem_size(qi);
  for (int which = 0; which < 2; ++which) {
    if ((which == 0 && !curr) || (which == 1 && !next)) continue;
    char *p = static_cast<char *>(which == 0 ? curr_data(qi) : next_data(qi)) - padX_[qi] * elem_size(qi);
    if (backend_ == Backend::Host) {
      std::memset(p, v, size_t(bytes));
    } else {
      set_device();
      HIP_CHECK(hipMemset(p, v, size_t(bytes)));
      HIP_CHECK(hipDeviceSynchronize());
    }
  }
}

} // namespace stencil
