#pragma once
// Compute kernels of the reference apps, written for CDNA4.
// Reference kernels:
//   Jacobi3D  init_kernel / stencil_kernel (6-neighbour mean + hot/cold spheres)   bin/jacobi3d.cu:18-87
//   Astaroth  init_kernel (sin wave, halo -10) / stencil_kernel (6-neighbour mean)  bin/astaroth_sim.cu:14-83
// The device kernel is a 2.5D z-march: each lane owns one 16-B x-chunk (4 fp32 / 2 fp64) of TY consecutive rows and
// walks z keeping planes z-1, z, z+1 in registers, so every interior cell is read from HBM ~once per sweep
// (y-halo rows are shared through L1/L2 by the 4 waves of a block, x-neighbours come from adjacent lanes by
// ds_bpermute). Blocks are remapped XCD-aware so y/z-adjacent tiles share an XCD's L2. Summation order and the
// division by 6 are the reference's, so results are bitwise identical to a sequential fp32 evaluation.
#include <cstdint>
#include <vector>

#include "stencil/core/geometry.hpp"
#include "stencil/domain/local_domain.hpp"

namespace stencil {

enum class StencilKind : int {
  Jacobi = 0,   // sum order +x,-x,+y,-y,+z,-z then /6, hot/cold spheres
  Astaroth = 1, // sum order -x,-y,-z,+x,+y,+z then /6
};

struct Spheres {
  bool enabled = false;
  Dim3 hot, cold;     // global coordinates of the sphere centres
  int64_t radius = 0; // cell is inside iff floor(sqrt(|p-c|^2)) <= radius  <=>  |p-c|^2 < (radius+1)^2
  // reference placement (bin/jacobi3d.cu:45-50) for a global compute region
  static Spheres jacobi(const Rect3 &cReg) {
    Spheres s;
    s.enabled = true;
    s.hot = Dim3(cReg.lo.x + (cReg.hi.x - cReg.lo.x) / 3, (cReg.lo.y + cReg.hi.y) / 2, (cReg.lo.z + cReg.hi.z) / 2);
    s.cold = Dim3(cReg.lo.x + (cReg.hi.x - cReg.lo.x) * 2 / 3, (cReg.lo.y + cReg.hi.y) / 2, (cReg.lo.z + cReg.hi.z) / 2);
    s.radius = (cReg.hi.x - cReg.lo.x) / 10;
    return s;
  }
};

struct StencilTune {
  // 2 (default): LDS-shared y-halo kernel with 2 planes of z lookahead (every row load has a whole z step to land;
  //    3/4: 3/4 planes), 0: LDS kernel with 1 plane (the loads are consumed in the step that issues them),
  //    1: register-only kernel. 512^3 fp32 on one MI355X: 201 us (v2) vs 212 us (v0) per sweep.
  int variant = 2;
  // variant kMfma: the x line update on the matrix cores (stencil7_mfma.hip; fp32 Jacobi, for counter comparison)
  static constexpr int kMfma = 8;
  int ty = 2;     // rows per lane (variant 0: 2/4/8, variant 1: 4/8)
  int zchunk = 0; // planes per block (0 = auto: exactly one round of resident blocks)
  int nw = 8;     // waves per block stacked in y (deep-lookahead variants: 4/8/16)
  int x3sched = 1;        // fused triples: 0 = the pairs' lockstep schedule, 1 = lockstep over the most row groups
  int x3parts = 0;        // fused triples, x3sched 1: lockstep z parts per row group (0 = the cost model's choice)
  // fused triples (Jacobi): extra weight of a sphere-crossing row-plane when the lockstep z parts are cut per row group
  // and the leftover groups planned (0: equal parts). 0.3 was best with equal leftover slices, 0.6 with levelled
  // slices (x3left 1, profiles/r6/r6z), 0.45 with the second lockstep phase (x3left 2 / 3: steady-state 512^3 triple
  // 226.1 us vs 228.2 at 0.3 and 228.1 at 0.6, driver command 1613-1633 Gcells/s, profiles/r6/r6ad)
  float x3sphw = 0.45f;
  float x2sphw = 0.15f;   // fused pairs (Jacobi, row / col2 kernels): sphere weight of the z parts (r5/at, r5/au)
  bool x3sphchunk = true; // fused triples (Jacobi): test each sphere only on the lane chunks its x range reaches
  // fused triples, lockstep parts: the row groups beyond the parts' (leftover groups) as second segments. 0 = equal
  // slices; 1 = slices levelling each block against the blocks whose parts cost more (sphere-crossing groups);
  // 2 = a second lockstep phase (every leftover group in K parts of common z bounds, blocks binned by their parts'
  // cost); 3 = whichever of 1 / 2 the host's step estimate prefers, with the number of parts chosen the same way
  int x3left = 3;
  bool x2early = true;    // fused pairs (row / col2 kernels): publish the src and u1 rows right after the u1 update
                          // (row kernel 208.6 vs 216.6 us per pair, col2 226.9 vs 234.1)
  // fused pairs of fp32 sub-domains: one wave per whole 512-cell periodic row (x wrapped in-kernel and 512 cells
  // long; x-neighbours and the wrap by DPP lane rotates, stencil7x2_row_kernel), or 512-cell columns (x a whole
  // number of 512-cell columns: two 16-B chunks per lane, only the column ends from outside the wave,
  // stencil7x2_col2_kernel). 0 = always the 256-cell column kernel
  int x2row = 1;
  // fused-pair work split: 1 (default) = one block per resident slot, each taking an equal share of the
  // (column, plane) space (one or two z segments): no partly empty last round and the fewest warm-up planes;
  // 0 = fixed z-chunks per block column (zchunk / auto)
  int x2sched = 1;
  // fused-pair column order: 1 = x-major (x-adjacent columns of a y range on one XCD), 0 = y-major. One MI355X:
  // 512^3 equal within noise (944-965 Gcells/s either way); 645/813/1024-wide shapes 2-3 % faster y-major
  int x2xfast = 0;
  // CUs an overlapped fused-pair interior sweep leaves free for the exchange kernels of the comm stream (balanced
  // segment mode: the grid is that many blocks short of the resident slots); reserveCUs is what one launch uses
  int x2reserve = 8;
  int reserveCUs = 0;
  // whole-row fused pairs with fewer resident blocks than 4 per row group (CUs reserved for the transports): four
  // blocks per column march lockstep z quarters, so y-adjacent blocks share their halo rows in L2 (512^3 local
  // interior beside the slab kernels 276 -> 252 us); false = the balanced (column, plane) split
  bool x2lockstep = true;
  // overlapped fused pairs: the z slabs of periodic 512-cell rows go through the whole-row kernel with the slab as its
  // z chunk (true) or through the thin slab kernel (false); both time the same within 2 % (r2s3)
  bool zslabRow = true;
  bool xcdRemap = true;
  bool nontemporal = true;
  // reverse the z-march of every block on odd buffer parities: each step then starts on the planes the previous
  // step wrote last, which are still in the MALL / L2
  // flip the z-march direction every pair (each sweep starts on the planes the previous one wrote last). r2s3, rows
  // 64-B aligned: -3 % (1164 vs 1202); r4, rows on whole 128-B lines: +2-6 % at 512^3 (interleaved bench.py
  // 1276-1290 vs 1256-1272, shape sweep 1321 / 1392 vs 1247 / 1311), +3-4 % at 645x645x323 and 1024x512x256, neutral
  // at 813-cell rows and fp64 (profiles/r4/q, profiles/r4/r): on
  bool alternateZ = true;
  // bitmask of axes (1 = x, 2 = y, 4 = z) along which the sub-domain is its own periodic
  // neighbour and the kernels read the periodic image in place of the halo (StencilModel sets it together with
  // DistributedDomain::exchange_async(.., skipWrapped), which then skips those same-GPU self copies). Needs the
  // region to span the whole compute region along wrapped axes, and for x an extent that is a multiple of the
  // 16-B chunk (fused pairs: >= 2 chunks). Fused pairs: stencil7x2_wrappable_axes; single steps (stencil7_apply):
  // stencil7_wrappable_axes. 0 = read halos.
  int wrap = 0;
  // pipelined pairs (StencilModel overlap mode 3; run-time state, not configuration): the whole-row kernel adds the
  // number of cells it has written in the first / last `publishDepth` z planes of the region to *publish (device
  // word, system-scope release after each such plane), so a gated exchange (DistributedDomain::set_send_gate) packs
  // the boundary planes while the rest of the sweep is still running. Other fused-pair kernels refuse it.
  uint64_t *publish = nullptr;
  // measurement: stencil7x3 writes every block's start / end wall clock (2 x uint64 per block) here when set
  uint64_t *blockClock = nullptr;
  int publishDepth = 0;
};
// the whole-row fused-pair kernel (the one that can publish its boundary planes) takes this region
bool stencil7x2_row_kernel_used(const LocalDomain &dom, int64_t qi, const Rect3 &region, const StencilTune &tune);
// axes (mask as StencilTune::wrap) the fused-pair kernels can wrap in-kernel for this quantity's layout; x2row as
// StencilTune::x2row (0: no whole-row kernel, so ragged x extents are not wrappable)
int stencil7x2_wrappable_axes(const LocalDomain &dom, int64_t qi, int x2row = 1);

// Halo forwarding: the producer writes its neighbours' halos. For every direction whose receiving halo lives in a
// sub-domain this process can store into directly (same GPU, or a P2P-mapped peer GPU over xGMI), the stencil
// kernel also stores each boundary output cell into the receiver's *next* buffer (the one that becomes curr after
// swap). A step is then one kernel per sub-domain (plus a small copy for receivers with a different layout): no
// pack, no separate exchange, and the halos of the new curr are valid when the step retires. Replaces the reference's separate exchange() for the Kernel/PeerCopy methods
// (reference tx_cuda.cuh:68-95 multi_translate, :141-162 peer copy).
struct ForwardTarget {
  Dim3 dir;                   // send direction
  const LocalDomain *dst;     // receiving sub-domain (same process)
  Dim3 offset;                // dst raw coordinate = src raw coordinate + offset
};

class HaloForwarder {
public:
  // per buffer parity (the receivers' next buffers alternate with swap()): an in-kernel store offset for every
  // receiver that shares this sub-domain's pitches, and a copy plan (run right after the kernel) for the others
  // (e.g. x neighbours of a different x size in an uneven partition). `targets` come from
  // DistributedDomain::forward_targets.
  HaloForwarder(const LocalDomain &src, int64_t qi, const std::vector<ForwardTarget> &targets);
  ~HaloForwarder();
  HaloForwarder(const HaloForwarder &) = delete;
  HaloForwarder &operator=(const HaloForwarder &) = delete;
  // cells within wm[a] of the low face send along -a, within wp[a] of the high face along +a
  const int *wm() const { return wm_; }
  const int *wp() const { return wp_; }
  int num_targets() const { return n_; }
  uint32_t mask(int parity) const { return mask_[parity]; }              // directions stored by the kernel
  int64_t delta(int parity, int k) const { return delta_[parity][k]; }   // element offset from the output cell
  bool has_rest() const { return hasRest_; }
  // copy the messages the kernel does not store (after the kernel, same stream)
  void forward_rest(int parity, hipStream_t stream) const;
  // can the forwarding kernel handle this sub-domain (aligned vector layout, fp32/fp64, sizes >= slab widths)?
  static bool supported(const LocalDomain &dom, int64_t qi);

private:
  int wm_[3] = {0, 0, 0}, wp_[3] = {0, 0, 0};
  int n_ = 0;
  int dev_ = -1;
  uint32_t mask_[2] = {0, 0};
  int64_t delta_[2][27] = {};
  CopyPlan rest_[2];
  bool hasRest_ = false;
};

// The host plan of a whole-row fused-triple sweep (stencil7x3's lockstep schedule, as apply runs it for a sub-domain
// of `size` cells with the reference's spheres for Jacobi, on `slots` resident blocks): for tests and tools, no GPU
struct X3PlanInfo {
  int parts = 0, blocks = 0, groups = 0, lockstepGroups = 0, rounds = 0;
  bool tabled = false;     // second segments from l0 / l1 / odd (leftover (column, plane) offsets), else equal slices
  double steps = 0;        // estimated steps of the longest block
  std::vector<int> zb;     // per lockstep group its parts - 1 z bounds (empty: equal parts)
  std::vector<int> l0, l1; // per block: its leftover slice
  std::vector<int> odd;    // per block: the slice's march direction bit
};
X3PlanInfo stencil7x3_plan(const Dim3 &size, bool jacobi, const StencilTune &tune, int slots = 256);
// dst(region) = stencil(src) for one quantity of one LocalDomain. `region` is in global coordinates and must lie in
// the domain's compute region; face radii must be >= 1. `currIsSrc` selects curr->next (true) or next->curr.
// With `fwd`, region must be the whole compute region and the output is also forwarded into the receivers' halos.
void stencil7_apply(const LocalDomain &dom, int64_t qi, const Rect3 &region, StencilKind kind, const Spheres &sph,
                    hipStream_t stream, const StencilTune &tune = StencilTune(), const HaloForwarder *fwd = nullptr);
// Two fused steps (temporal blocking): dst(region) = S(S(src)), bitwise equal to two single steps. Needs halos of
// depth 2 on the faces and 1 on the edges (Radius::face_edge_corner(2, 1, 0) or more) valid in src, a device
// fp32/fp64 quantity and the aligned layout (stencil7x2_supported). Reads src once and writes dst once per two steps.
bool stencil7x2_supported(const LocalDomain &dom, int64_t qi);
void stencil7x2_apply(const LocalDomain &dom, int64_t qi, const Rect3 &region, StencilKind kind, const Spheres &sph,
                      hipStream_t stream, const StencilTune &tune = StencilTune());
// Three fused steps: dst = S(S(S(src))) on the whole compute region, bitwise equal to three single steps. x either
// wraps in-kernel (tune.wrap & 1: fp32 rows of exactly 512 cells) or is read from 3-deep halos (fp32 x a multiple of
// 512, fp64 of 256; faces, edges and corners exchanged); y / z wrap in-kernel or read 3-deep halos.
// Returns false (nothing launched) when this layout / region / tune is not supported.
bool stencil7x3_supported(const LocalDomain &dom, int64_t qi, const Rect3 &region, const StencilTune &tune);
bool stencil7x3_apply(const LocalDomain &dom, int64_t qi, const Rect3 &region, StencilKind kind, const Spheres &sph,
                      hipStream_t stream, const StencilTune &tune);
// S o S on several small regions (the exterior slabs of an overlapped fused pair), one thread per cell
void stencil7x2_apply_regions(const LocalDomain &dom, int64_t qi, const std::vector<Rect3> &regions, StencilKind kind,
                              const Spheres &sph, hipStream_t stream, int wrap = 0);
// S o S on the compute region minus `interior` (the exterior of an overlapped fused pair): z slabs and y slabs by
// the sweep kernel (6 waves per block for 2-row slabs), thin x slabs by a lanes-on-rows kernel
void stencil7x2_apply_exterior(const LocalDomain &dom, int64_t qi, const Rect3 &interior, StencilKind kind,
                               const Spheres &sph, hipStream_t stream, const StencilTune &tune = StencilTune());
// Lockstep block schedule of the whole-row / 512-cell-column fused pairs: `slots` resident blocks, `cols` row
// groups (8 output rows of one column strip each), `nz` planes. P blocks per row group march P z parts side by side (y-adjacent blocks on one XCD, so their
// shared y-halo rows meet in L2): quarters (P = 4) over the first slots / 4 row groups with the rest as short
// second segments, or P = slots / cols over every row group when the grid has fewer than slots / 4 row groups or
// the row groups divide the slots evenly; rounds of whole columns when there are more row groups than slots
// (813x407x407: 51 groups, 5 parts, 847 -> 910-917 Gcells/s; 645x323x645: 41 groups, 6 parts, 847 -> 1067-1072).
// Whole columns over fewer slots instead of quarters plus leftovers lose (645x645x323, 81 groups: 3 parts on 243
// blocks 930-946 vs 994-1001; profiles/r3/s3/ab_lockstep_parts.txt). parts == 0: no lockstep (parts under 16
// planes, or nz < 64): balanced split.
struct X2Schedule {
  int parts = 0;
  int64_t blocks = 0;
  int rounds = 1; // > 1: block b marches part b / cm of columns b % cm, b % cm + cm, ... (cm = blocks / parts) in
                  // step with the others; parts 1 = whole columns
};
inline X2Schedule x2_lockstep_schedule(int64_t slots, int64_t cols, int64_t nz) {
  X2Schedule r;
  if (slots < 4 || cols < 1) return r;
  if (cols > slots) {
    // more row groups than blocks (fp64 1024^3 as 256-cell columns: 4 x 128 groups): rounds of whole columns, every
    // block on one column per round, y-adjacent columns side by side (quarters plus leftovers would run most
    // columns as balanced second segments)
    if (nz < 16) return r;
    r.rounds = int((cols + slots - 1) / slots);
    r.parts = 1;
    r.blocks = (cols + r.rounds - 1) / r.rounds;
    return r;
  }
  // whole columns when they divide the slots evenly (1024x512x256 on the 512-cell column kernel: 128 columns, P = 2)
  const int64_t P = (slots / 4 > cols || slots % cols == 0) ? slots / cols : 4;
  const int64_t cm = cols < slots / P ? cols : slots / P;
  if (cm < 1 || nz < 64 || nz / P < 16) return r;
  r.parts = int(P);
  r.blocks = P * cm;
  if (P == 4 && cm < cols && cols % 2 == 0) {
    // quarters over slots / 4 row groups leave the rest to balanced second segments; two rounds of P2 parts over
    // half the row groups each keep every segment in lockstep when they fill 15 / 16 of the slots in both rounds
    // (813x813x204: 102 groups = 2 rounds x 51 groups x 5 parts on 255 blocks, 928-931 -> 970-971 Gcells/s; an odd
    // count idles blocks in the second round: 645x645x323, 81 groups as 2 x 41 x 6, 1034 -> 1009-1018, not taken;
    // profiles/r3/s3/ab_rounds_parts.txt)
    const int64_t ch = cols / 2, P2 = slots / ch;
    if (P2 >= 2 && nz / P2 >= 16 && 16 * P2 * ch >= 15 * slots) {
      r.parts = int(P2);
      r.blocks = P2 * ch;
      r.rounds = 2;
    }
  }
  return r;
}

// axes (mask as StencilTune::wrap) stencil7_apply can wrap in-kernel for this quantity's layout: with tune.wrap set
// the single step reads the periodic image along those axes instead of the halo (the region must span them)
int stencil7_wrappable_axes(const LocalDomain &dom, int64_t qi);
// MFMA variant of the single step (fp32 Jacobi; StencilTune::variant == kMfma routes stencil7_apply here)
bool stencil7_mfma_supported(const LocalDomain &dom, int64_t qi);
void stencil7_mfma_apply(const LocalDomain &dom, int64_t qi, const Rect3 &region, StencilKind kind, const Spheres &sph,
                         hipStream_t stream, const StencilTune &tune = StencilTune());
// same for several regions in one call (e.g. the exterior slabs)
void stencil7_apply_regions(const LocalDomain &dom, int64_t qi, const std::vector<Rect3> &regions, StencilKind kind,
                            const Spheres &sph, hipStream_t stream, const StencilTune &tune = StencilTune());

// Jacobi init: curr = 0.5 on `region` (reference bin/jacobi3d.cu:18-29)
void jacobi_init(const LocalDomain &dom, int64_t qi, const Rect3 &region, hipStream_t stream);
// Astaroth init: interior = sin(2*pi/period*(origin+x+y+z)) (x,y,z raw indices), halo = -10 (astaroth_sim.cu:14-61)
void astaroth_init(const LocalDomain &dom, int64_t qi, double period, hipStream_t stream);
// fill every cell of the full region (halo included) of curr with a value
void fill_value(const LocalDomain &dom, int64_t qi, double value, bool curr, hipStream_t stream);

} // namespace stencil
