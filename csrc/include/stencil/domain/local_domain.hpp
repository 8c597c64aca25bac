#pragma once
// LocalDomain: one sub-domain (interior + halo) of every quantity, on one GPU or in host memory.
// Parity: reference include/stencil/local_domain.cuh:33-349, src/local_domain.cu:1-168
//   add_data / set_radius / realize / get_curr / get_next / accessors / halo_pos / halo_extent /
//   halo_coords / halo_bytes / raw_size / size / origin / gpu / swap / region_to_host / interior_to_host /
//   quantity_to_host
// MI355X layout: the x pitch is padded so the first interior x of every row is 128-B aligned (one
// L2 line; set_interior_align(64) for the rounds-1-3 sector alignment) and every row starts on a 128-B line; y/z are
// unpadded. Halo-aligned x (set_x_halo_align, x halos of at most 48 B):
// the interior starts 16-B aligned inside the row's first 64-B sector, with the -x halo directly in front of it in
// that same sector and the +x halo directly behind the interior's last cells, so an x-face copy touches one sector
// per row end instead of two (the stencil kernels' 16-B chunk grid still starts at the interior; a row then spans
// one more sector). A 128-B guard before the first row keeps reads left of raw x = 0 inside the allocation. `raw_size()` keeps the reference's logical meaning
// (interior + halo), `pitch()` is the physical stride. Pointers are swapped on the host only: kernels receive
// pointers by value, so swap() needs no device-side pointer-table upload (reference local_domain.cu:41-54
// issues a synchronous cudaMemcpy there).
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "stencil/core/geometry.hpp"
#include "stencil/kernels/copy.hpp"
#include "stencil/rt/logging.hpp"

namespace stencil {

enum class Backend { Host = 0, Device = 1 };

// element type tag (used by Python views and the ParaView writer)
enum class DType : int { Bytes = 0, F32 = 1, F64 = 2, I32 = 3, I64 = 4, U8 = 5, I8 = 6, F16 = 7, BF16 = 8, U32 = 9, U64 = 10 };
template <typename T> constexpr DType dtype_of() { return DType::Bytes; }
template <> constexpr DType dtype_of<float>() { return DType::F32; }
template <> constexpr DType dtype_of<double>() { return DType::F64; }
template <> constexpr DType dtype_of<int32_t>() { return DType::I32; }
template <> constexpr DType dtype_of<int64_t>() { return DType::I64; }
template <> constexpr DType dtype_of<uint8_t>() { return DType::U8; }
template <> constexpr DType dtype_of<int8_t>() { return DType::I8; }
template <> constexpr DType dtype_of<uint32_t>() { return DType::U32; }
template <> constexpr DType dtype_of<uint64_t>() { return DType::U64; }
template <> constexpr DType dtype_of<char>() { return DType::I8; }

template <typename T> struct DataHandle {
  int64_t id_;
  std::string name_;
  explicit DataHandle(int64_t i = -1, const std::string &name = "") : id_(i), name_(name) {}
  int64_t id() const { return id_; }
  const std::string &name() const { return name_; }
};

class LocalDomain {
public:
  LocalDomain(const Dim3 &sz, const Dim3 &origin, int dev, Backend backend = Backend::Device);
  ~LocalDomain();
  LocalDomain(const LocalDomain &) = delete;
  LocalDomain &operator=(const LocalDomain &) = delete;
  LocalDomain(LocalDomain &&o) noexcept;
  LocalDomain &operator=(LocalDomain &&) = delete;

  // ---- configuration (before realize) ----
  int64_t add_data(int64_t elemSize, const std::string &name = "", DType dtype = DType::Bytes);
  template <typename T> DataHandle<T> add_data(const std::string &name = "") {
    return DataHandle<T>(add_data(int64_t(sizeof(T)), name, dtype_of<T>()), name);
  }
  void set_radius(int64_t r) { radius_ = Radius::constant(r); }
  void set_radius(const Radius &r) { radius_ = r; }
  void set_padding(bool pad) { pad_ = pad; }
  void set_x_halo_align(bool on) { xHaloAlign_ = on; }
  // byte alignment of the first interior x of every row: 128 (default) = one L2 line, so a 512-cell fp32 row spans 16
  // lines instead of 17 (one MI355X, fused pairs at 512^3: 1150-1194 -> 1285-1287 Gcells/s, FETCH_SIZE 296 -> 279 MB
  // per pair; profiles/r4/i/); 64 = one sector (rounds 1-3)
  void set_interior_align(int64_t bytes) {
    STENCIL_REQUIRE(bytes == 64 || bytes == 128, "interior alignment must be 64 or 128 B");
    interiorAlign_ = bytes;
  }
  int64_t interior_align() const { return interiorAlign_; }
  // extra 128-B lines appended to every row's pitch (measurement knob: row / plane strides vs HBM channel mapping)
  void set_row_pad_lines(int n) { rowPadLines_ = n; }
  int row_pad_lines() const { return rowPadLines_; }
  bool x_halo_align() const { return xHaloAlign_; }
  // shared halo lines: the row pitch is the raw row rounded up to whole interior-alignment units
  // (512^3 fp32 radius 2: 17 lines of 128 B instead of 18), so row r's +x halo and row r+1's -x halo sit in ONE line
  // -- the line between row r's last and row r+1's first interior line. A row's raw cells then reach into the next
  // row's front padding (never into its raw cells); x-face self copies write each shared line from one item (both
  // halos: make_copy_plan pairs them), i.e. one written line per row instead of two. Needs the padded layout, the
  // interior on an alignment unit and x halos that fit one unit together; ignored with the halo-aligned x layout.
  void set_shared_halo_line(bool on) { sharedLine_ = on; }
  bool shared_halo_line() const { return sharedLine_ && sharedActive_; }
  void realize();
  bool realized() const { return realized_; }

  // ---- geometry ----
  const Dim3 &size() const { return sz_; }
  const Dim3 &origin() const { return origin_; }
  const Radius &radius() const { return radius_; }
  int gpu() const { return dev_; }
  Backend backend() const { return backend_; }
  int64_t num_data() const { return int64_t(elemSize_.size()); }
  int64_t elem_size(int64_t qi) const { return elemSize_.at(size_t(qi)); }
  DType dtype(int64_t qi) const { return dtype_.at(size_t(qi)); }
  const std::string &name(int64_t qi) const { return names_.at(size_t(qi)); }
  void set_name(int64_t qi, const std::string &n) { names_.at(size_t(qi)) = n; }

  // logical allocation extent (interior + halo), reference raw_size()
  Dim3 raw_size() const {
    return Dim3(sz_.x + radius_.x(-1) + radius_.x(1), sz_.y + radius_.y(-1) + radius_.y(1),
                sz_.z + radius_.z(-1) + radius_.z(1));
  }
  // physical stride in elements of quantity qi: (padded x pitch, raw y, raw z)
  Dim3 pitch(int64_t qi) const { return Dim3(pitchX_.at(size_t(qi)), raw_size().y, raw_size().z); }
  // elements of padding in front of raw x = 0 in every row
  int64_t pad_x(int64_t qi) const { return padX_.at(size_t(qi)); }
  // elements in front of raw x = 0 that a kernel may read (ignoring the values) without leaving the allocation:
  // the row padding, plus the guard before the first row (halo-aligned layout)
  int64_t front_slack(int64_t qi) const { return padX_.at(size_t(qi)) + guard_ / elem_size(qi); }
  // raw x (exclusive, from a row's raw x = 0) up to which a kernel may READ in any row without leaving the allocation
  // (values beyond the row's raw cells are ignored): the end of the row's own pitch block, and with shared halo
  // lines the end of the next row's front padding (the last row of a buffer has an allocated tail for it)
  int64_t row_limit(int64_t qi) const { return pitchX_.at(size_t(qi)) - (shared_halo_line() ? 0 : padX_.at(size_t(qi))); }
  // bytes of one curr (or next) buffer of quantity qi
  int64_t buffer_bytes(int64_t qi) const;

  Rect3 get_compute_region() const { return Rect3(origin_, origin_ + sz_); }
  Rect3 get_full_region() const {
    return Rect3(origin_ - Dim3(radius_.x(-1), radius_.y(-1), radius_.z(-1)),
                 origin_ + sz_ + Dim3(radius_.x(1), radius_.y(1), radius_.z(1)));
  }
  // position (relative to raw [0,0,0]) of the halo (halo=true) or of the interior slab that feeds the neighbour
  // (halo=false) on the `dir` side. dir = 0 gives the interior origin.
  Dim3 halo_pos(const Dim3 &dir, bool halo) const;
  Rect3 halo_coords(const Dim3 &dir, bool halo) const;
  static Dim3 halo_extent(const Dim3 &dir, const Dim3 &sz, const Radius &radius) {
    return Dim3(dir.x == 0 ? sz.x : radius.x(int(dir.x)), dir.y == 0 ? sz.y : radius.y(int(dir.y)),
                dir.z == 0 ? sz.z : radius.z(int(dir.z)));
  }
  Dim3 halo_extent(const Dim3 &dir) const { return halo_extent(dir, sz_, radius_); }
  int64_t halo_bytes(const Dim3 &dir, int64_t qi) const { return elem_size(qi) * halo_extent(dir).flatten(); }

  // ---- data ----
  void *curr_data(int64_t qi) const { return curr_.at(size_t(qi)); }
  void *next_data(int64_t qi) const { return next_.at(size_t(qi)); }
  template <typename T> T *get_curr(const DataHandle<T> &h) const { return static_cast<T *>(curr_data(h.id_)); }
  template <typename T> T *get_next(const DataHandle<T> &h) const { return static_cast<T *>(next_data(h.id_)); }
  template <typename T> Accessor<T> get_curr_accessor(const DataHandle<T> &h) const {
    return Accessor<T>(get_curr(h), accessor_origin(), pitch(h.id_));
  }
  template <typename T> Accessor<T> get_next_accessor(const DataHandle<T> &h) const {
    return Accessor<T>(get_next(h), accessor_origin(), pitch(h.id_));
  }
  // global coordinate of raw element [0,0,0]
  Dim3 accessor_origin() const { return origin_ - Dim3(radius_.x(-1), radius_.y(-1), radius_.z(-1)); }

  // strided view of quantity qi (curr or next) starting at raw position `pos`
  StridedBox box(int64_t qi, bool curr, const Dim3 &pos) const;

  // swap curr and next of every quantity (host pointers only)
  void swap();
  int parity() const { return parity_; }

  // ---- host transfer (synchronous) ----
  std::vector<unsigned char> region_to_host(const Dim3 &pos, const Dim3 &ext, int64_t qi, bool curr = true) const;
  void region_from_host(const Dim3 &pos, const Dim3 &ext, int64_t qi, const void *src, bool curr = true);
  std::vector<unsigned char> interior_to_host(int64_t qi) const {
    return region_to_host(halo_pos(Dim3(0, 0, 0), true), sz_, qi);
  }
  std::vector<unsigned char> quantity_to_host(int64_t qi) const { return region_to_host(Dim3(0, 0, 0), raw_size(), qi); }
  // fill every byte of both buffers of quantity qi (e.g. NaN poisoning for race canaries)
  void fill_bytes(int64_t qi, uint8_t v, bool curr, bool next);

  void set_device() const;

private:
  Dim3 sz_, origin_;
  Radius radius_;
  int dev_;
  Backend backend_;
  bool pad_ = true;
  bool xHaloAlign_ = false;
  bool sharedLine_ = false, sharedActive_ = false;
  int64_t interiorAlign_ = 128;
  int rowPadLines_ = 0;
  int64_t guard_ = 0; // bytes before the first row of every buffer (halo-aligned layout)
  bool realized_ = false;
  int parity_ = 0;
  std::vector<int64_t> elemSize_;
  std::vector<DType> dtype_;
  std::vector<std::string> names_;
  std::vector<int64_t> pitchX_, padX_;
  std::vector<int64_t> tailX_; // elements allocated after the last pitch block (shared halo lines)
  std::vector<void *> base_[2]; // allocations
  std::vector<void *> curr_, next_;
  void free_all();
};

} // namespace stencil
