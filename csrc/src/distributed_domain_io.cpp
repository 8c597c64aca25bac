// DistributedDomain output and restart: ParaView CSV dumps (reference src/stencil.cu:866-939) and checkpoints (no
// reference counterpart), split out of distributed_domain.cpp.
#include "stencil/domain/distributed_domain.hpp"

#include <hip/hip_runtime_api.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "stencil/rt/hip_check.hpp"
#include "stencil/rt/trace.hpp"

namespace stencil {

// ------------------------------------------------------------------------------------------------
// ParaView CSV (reference src/stencil.cu:866-939), quantity names preserved
// ------------------------------------------------------------------------------------------------
void DistributedDomain::write_paraview(const std::string &prefix, bool zeroNaNs) {
  TraceRange tr("write_paraview");
  if (backend_ == Backend::Device) sync_exchange();
  for (size_t di = 0; di < domains_.size(); ++di) {
    const LocalDomain &d = domains_[di];
    const int64_t id = int64_t(rank()) * int64_t(domains_.size()) + int64_t(di);
    const std::string path = prefix + "_" + std::to_string(id) + ".txt";
    std::vector<std::vector<unsigned char>> qs;
    for (int64_t q = 0; q < d.num_data(); ++q) qs.push_back(d.interior_to_host(q));
    FILE *f = std::fopen(path.c_str(), "w");
    STENCIL_REQUIRE(f, "cannot open " << path);
    std::fprintf(f, "Z,Y,X");
    for (int64_t q = 0; q < d.num_data(); ++q) {
      std::string n = d.name(q);
      if (n.empty()) n = "data" + std::to_string(q);
      std::fprintf(f, ",%s", n.c_str());
    }
    std::fprintf(f, "\n");
    const Dim3 sz = d.size(), o = d.origin();
    std::string line;
    char buf[64];
    for (int64_t z = 0; z < sz.z; ++z)
      for (int64_t y = 0; y < sz.y; ++y)
        for (int64_t x = 0; x < sz.x; ++x) {
          line.clear();
          std::snprintf(buf, sizeof(buf), "%ld,%ld,%ld", long(o.z + z), long(o.y + y), long(o.x + x));
          line += buf;
          const int64_t li = x + sz.x * (y + sz.y * z);
          for (int64_t q = 0; q < d.num_data(); ++q) {
            const unsigned char *p = qs[q].data() + li * d.elem_size(q);
            switch (d.dtype(q)) {
            case DType::F64: {
              double v;
              std::memcpy(&v, p, 8);
              if (zeroNaNs && std::isnan(v)) v = 0;
              std::snprintf(buf, sizeof(buf), ",%f", v);
              break;
            }
            case DType::I32: {
              int32_t v;
              std::memcpy(&v, p, 4);
              std::snprintf(buf, sizeof(buf), ",%d", v);
              break;
            }
            case DType::I64: {
              int64_t v;
              std::memcpy(&v, p, 8);
              std::snprintf(buf, sizeof(buf), ",%ld", long(v));
              break;
            }
            default: {
              if (d.elem_size(q) == 8) {
                double v;
                std::memcpy(&v, p, 8);
                if (zeroNaNs && std::isnan(v)) v = 0;
                std::snprintf(buf, sizeof(buf), ",%f", v);
              } else {
                float v = 0;
                std::memcpy(&v, p, std::min<int64_t>(4, d.elem_size(q)));
                if (zeroNaNs && std::isnan(v)) v = 0;
                std::snprintf(buf, sizeof(buf), ",%f", double(v));
              }
            }
            }
            line += buf;
          }
          line += "\n";
          std::fputs(line.c_str(), f);
        }
    std::fclose(f);
  }
}

} // namespace stencil

namespace stencil {

namespace {
struct CkptHeader {
  uint64_t magic;
  int64_t global[3];
  int64_t idx[3];
  int64_t origin[3];
  int64_t size[3];
  int64_t nq;
};
constexpr uint64_t kCkptMagic = 0x53544e434b505432ull; // "STNCKPT2"
} // namespace

void DistributedDomain::save_checkpoint(const std::string &prefix) const {
  STENCIL_REQUIRE(realized_, "save_checkpoint before realize");
  const_cast<DistributedDomain *>(this)->sync_exchange();
  for (size_t di = 0; di < domains_.size(); ++di) {
    const LocalDomain &d = domains_[di];
    const std::string path = prefix + "_" + std::to_string(rank()) + "_" + std::to_string(di) + ".ckpt";
    FILE *f = std::fopen(path.c_str(), "wb");
    STENCIL_REQUIRE(f, "cannot open " << path);
    const Dim3 idx = placement_->get_idx(rank(), int(di));
    CkptHeader h{kCkptMagic, {size_.x, size_.y, size_.z}, {idx.x, idx.y, idx.z}, {d.origin().x, d.origin().y, d.origin().z},
                 {d.size().x, d.size().y, d.size().z}, d.num_data()};
    std::fwrite(&h, sizeof(h), 1, f);
    for (int64_t q = 0; q < d.num_data(); ++q) {
      const int64_t es = d.elem_size(q);
      std::fwrite(&es, sizeof(es), 1, f);
    }
    for (int64_t q = 0; q < d.num_data(); ++q) {
      auto v = d.interior_to_host(q);
      std::fwrite(v.data(), 1, v.size(), f);
    }
    std::fclose(f);
  }
  pg_->barrier();
}

void DistributedDomain::load_checkpoint(const std::string &prefix) {
  STENCIL_REQUIRE(realized_, "load_checkpoint before realize");
  sync_exchange();
  for (size_t di = 0; di < domains_.size(); ++di) {
    LocalDomain &d = domains_[di];
    const std::string path = prefix + "_" + std::to_string(rank()) + "_" + std::to_string(di) + ".ckpt";
    FILE *f = std::fopen(path.c_str(), "rb");
    STENCIL_REQUIRE(f, "cannot open " << path);
    CkptHeader h{};
    STENCIL_REQUIRE(std::fread(&h, sizeof(h), 1, f) == 1 && h.magic == kCkptMagic, "bad checkpoint " << path);
    const Dim3 idx = placement_->get_idx(rank(), int(di));
    STENCIL_REQUIRE(h.global[0] == size_.x && h.global[1] == size_.y && h.global[2] == size_.z && h.idx[0] == idx.x &&
                        h.idx[1] == idx.y && h.idx[2] == idx.z && h.size[0] == d.size().x && h.size[1] == d.size().y &&
                        h.size[2] == d.size().z && h.nq == d.num_data(),
                    "checkpoint " << path << " does not match this decomposition");
    for (int64_t q = 0; q < d.num_data(); ++q) {
      int64_t es = 0;
      STENCIL_REQUIRE(std::fread(&es, sizeof(es), 1, f) == 1 && es == d.elem_size(q), "element size mismatch in " << path);
    }
    for (int64_t q = 0; q < d.num_data(); ++q) {
      std::vector<unsigned char> v(size_t(d.size().flatten() * d.elem_size(q)));
      STENCIL_REQUIRE(std::fread(v.data(), 1, v.size(), f) == v.size(), "truncated checkpoint " << path);
      d.region_from_host(d.halo_pos(Dim3(0, 0, 0), true), d.size(), q, v.data());
    }
    std::fclose(f);
  }
  pg_->barrier();
}

} // namespace stencil
