#pragma once
// Device helpers shared by the fused-pair kernels (stencil7x2.hip) and the whole-row single step (stencil7_row.hip):
// packed pairs, DPP lane shifts and rotates, reference-order six-term sums and the exact /6.
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

#include "stencil_common.hpp"

namespace stencil {

// Packed-math helpers. A wave64 fp32 VALU op covers 64 lanes x 1 value; v_pk_{add,mul,fma}_f32 cover 64 x 2 at the
// same issue cost, so rows are summed as pairs (2 pk ops per 4-float chunk per term). fp64 has no packed form: the
// pair type is then two scalar ops. IEEE per element, so results are bitwise those of the scalar code.
template <typename T> struct Pk;
template <> struct Pk<float> { typedef float t __attribute__((ext_vector_type(2))); };
template <> struct Pk<double> { typedef double t __attribute__((ext_vector_type(2))); };

// whole-wave lane shifts on the DPP path (a VALU mov, no LDS round trip as with ds_bpermute): lane i receives
// lane i-1 (wave_shr:1) / lane i+1 (wave_shl:1); the lanes shifted in from outside the wave get 0 and are replaced
// by the edge scalars
__device__ __forceinline__ int dpp_shr1(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x138, 0xf, 0xf, false); }
__device__ __forceinline__ int dpp_shl1(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x130, 0xf, 0xf, false); }
template <typename T> __device__ __forceinline__ T from_prev_lane(T v);
template <typename T> __device__ __forceinline__ T from_next_lane(T v);
template <> __device__ __forceinline__ float from_prev_lane<float>(float v) { return __int_as_float(dpp_shr1(__float_as_int(v))); }
template <> __device__ __forceinline__ float from_next_lane<float>(float v) { return __int_as_float(dpp_shl1(__float_as_int(v))); }
template <> __device__ __forceinline__ double from_prev_lane<double>(double v) {
  const int64_t b = __double_as_longlong(v);
  return __longlong_as_double(int64_t(uint32_t(dpp_shr1(int(b)))) | (int64_t(dpp_shr1(int(b >> 32))) << 32));
}
template <> __device__ __forceinline__ double from_next_lane<double>(double v) {
  const int64_t b = __double_as_longlong(v);
  return __longlong_as_double(int64_t(uint32_t(dpp_shl1(int(b)))) | (int64_t(dpp_shl1(int(b >> 32))) << 32));
}

// Six-term sums in the reference's order (sum6 in stencil_common.hpp), element-wise over a vector type. The fp32
// sums start from the first term instead of 0 + first term: the two differ only in the sign of an all-zero sum,
// and the exact /6 below maps both zeros to +0 as the 0-started sum does. fp64 keeps the 0 start.
template <typename T, int KIND, typename X>
__device__ __forceinline__ X sum6v(const X &vpx, const X &vmx, const X &vpy, const X &vmy, const X &vpz, const X &vmz) {
  X s;
  if constexpr (KIND == 0) {
    s = std::is_same<T, float>::value ? vpx : X(T(0)) + vpx;
    s += vmx;
    s += vpy;
    s += vmy;
    s += vpz;
    s += vmz;
  } else {
    s = std::is_same<T, float>::value ? vmx : X(T(0)) + vmx;
    s += vmy;
    s += vmz;
    s += vpx;
    s += vpy;
    s += vpz;
  }
  return s;
}
// exact element-wise /6 (div6): two FMAs around the reciprocal (fp32 packed); sums with 0 < |s| < 2^-100 (fp64:
// 2^-960), where the FMA form is not exact, take the true division in a branch no wave normally enters
template <typename T, typename X, int N> __device__ __forceinline__ X div6v(const X &s) {
  if constexpr (std::is_same<T, float>::value) {
    const X c = X(1.0f / 6.0f), six = X(6.0f);
    const X q0 = s * c;
    const X r = __builtin_elementwise_fma(-q0, six, s);
    X q = __builtin_elementwise_fma(r, c, q0);
    float m = __builtin_fabsf(s[0]);
#pragma unroll
    for (int e = 1; e < N; ++e) m = __builtin_fminf(m, __builtin_fabsf(s[e]));
    if (__builtin_expect(m < 0x1p-100f, 0)) {
#pragma unroll
      for (int e = 0; e < N; ++e)
        if (__builtin_fabsf(s[e]) < 0x1p-100f && s[e] != 0.0f) q[e] = s[e] / 6.0f;
    }
    return q;
  } else {
    // fp64: the same two FMAs around RN(1/6) (Markstein's corrected quotient; 1.2e9 random inputs, half of them
    // near multiples of 3, all equal to the IEEE quotient for |s| >= 2^-960: scripts/mi355x/lab/div6_fp64_check.cpp)
    // instead of the ~10-instruction division sequence; smaller sums (subnormal-range results) divide
    const X c = X(1.0 / 6.0), six = X(6.0);
    const X q0 = s * c;
    const X r = __builtin_elementwise_fma(-q0, six, s);
    X q = __builtin_elementwise_fma(r, c, q0);
    double m = __builtin_fabs(s[0]);
#pragma unroll
    for (int e = 1; e < N; ++e) m = __builtin_fmin(m, __builtin_fabs(s[e]));
    if (__builtin_expect(m < 0x1p-960, 0)) {
#pragma unroll
      for (int e = 0; e < N; ++e)
        if (__builtin_fabs(s[e]) < 0x1p-960 && s[e] != 0.0) q[e] = s[e] / 6.0;
    }
    return q;
  }
}

// calls f(integral_constant<I>) for I = 0, 1, ... while it returns true; true if all did
template <typename F, int... I> __device__ __forceinline__ bool run_phases(F &f, std::integer_sequence<int, I...>) {
  return (f(std::integral_constant<int, I>{}) && ...);
}

// wave rotates write every lane, so no old value: mov_dpp leaves it undefined (update_dpp(0, ...) cost a v_mov 0 per
// rotate) and lets the DPP combiner fold the rotate into its consumer
__device__ __forceinline__ float rot_prev(float v) { // lane i <- lane i-1, lane 0 <- lane 63 (wave_ror:1)
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x13C, 0xf, 0xf, false));
}
__device__ __forceinline__ float rot_next(float v) { // lane i <- lane i+1, lane 63 <- lane 0 (wave_rol:1)
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x134, 0xf, 0xf, false));
}

__device__ __forceinline__ double rot_prev(double v) { // fp64: both 32-bit halves rotated
  const int64_t b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp(int(b), 0x13C, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(int(b >> 32), 0x13C, 0xf, 0xf, false);
  return __longlong_as_double(int64_t(uint32_t(lo)) | (int64_t(hi) << 32));
}
__device__ __forceinline__ double rot_next(double v) {
  const int64_t b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp(int(b), 0x134, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(int(b >> 32), 0x134, 0xf, 0xf, false);
  return __longlong_as_double(int64_t(uint32_t(lo)) | (int64_t(hi) << 32));
}

} // namespace stencil
