// HBM bandwidth probe for the fused-pair kernel's access shape (lab, not part of the library).
// 512^3 fp32 fields (537 MB each). Prints one CSV line per variant: name,blocks,waves,us,TB/s (bytes read + written).
//   copy / write / read:   grid-stride float4 streams, 256 threads per block, plain or nontemporal stores
//   rows<NW,H,PF,NT>:      the fused pair's shape: one block per CU (NW waves), each wave streams whole 512-cell rows
//                          (H 16-B chunks per lane), PF rows of loads in flight, z-marching columns of NW rows
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                                                          \
  do {                                                                                                                 \
    hipError_t e_ = (x);                                                                                               \
    if (e_ != hipSuccess) {                                                                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                                   \
      std::exit(1);                                                                                                    \
    }                                                                                                                  \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT> __global__ __launch_bounds__(256) void k_copy(const f4 *__restrict__ s, f4 *__restrict__ d, long n) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += long(gridDim.x) * 256) {
    f4 v = s[i];
    if (NT)
      __builtin_nontemporal_store(v, d + i);
    else
      d[i] = v;
  }
}

template <bool NT> __global__ __launch_bounds__(256) void k_write(f4 *__restrict__ d, long n, float c) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += long(gridDim.x) * 256) {
    f4 v = {c, c + 1, c + 2, float(i)};
    if (NT)
      __builtin_nontemporal_store(v, d + i);
    else
      d[i] = v;
  }
}

__global__ __launch_bounds__(256) void k_read(const f4 *__restrict__ s, long n, float *out) {
  f4 acc = {0, 0, 0, 0};
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += long(gridDim.x) * 256) acc += s[i];
  if (acc.x + acc.y + acc.z + acc.w == 12345.f) out[0] = 1;
}

// rows: X = 512 cells (128 float4 per row = 2 chunks per lane), Y rows per plane, Z planes. Block b owns y rows
// [NW*(b % (Y/NW)), +NW) and z quarter b / (Y/NW) (so 4 * Y/NW blocks); wave w streams row y0+w through its planes.
template <int NW, int PF, bool NT>
__global__ __launch_bounds__(64 * NW, 1) void k_rows(const f4 *__restrict__ s, f4 *__restrict__ d, int Y, int Z,
                                                     int nq) {
  const int lane = threadIdx.x, w = threadIdx.y;
  const int cols = Y / NW;
  const int col = blockIdx.x % cols, q = blockIdx.x / cols;
  const int z0 = q * Z / nq, z1 = (q + 1) * Z / nq;
  const long row = long(col * NW + w) * 128;
  const long plane = long(Y) * 128;
  f4 a[PF + 1][2];
#pragma unroll
  for (int k = 0; k < PF; ++k) {
    const int z = z0 + k < z1 ? z0 + k : z1 - 1;
    a[k][0] = s[z * plane + row + lane];
    a[k][1] = s[z * plane + row + 64 + lane];
  }
  for (int z = z0; z < z1; z += PF + 1) {
#pragma unroll
    for (int k = 0; k <= PF; ++k) {
      const int zl = z + k + PF; // load PF ahead
      const int zc = zl < z1 ? zl : z1 - 1;
      a[(k + PF) % (PF + 1)][0] = s[zc * plane + row + lane];
      a[(k + PF) % (PF + 1)][1] = s[zc * plane + row + 64 + lane];
      if (z + k < z1) {
        f4 *o = d + (z + k) * plane + row;
        if (NT) {
          __builtin_nontemporal_store(a[k % (PF + 1)][0], o + lane);
          __builtin_nontemporal_store(a[k % (PF + 1)][1], o + 64 + lane);
        } else {
          o[lane] = a[k % (PF + 1)][0];
          o[64 + lane] = a[k % (PF + 1)][1];
        }
      }
    }
  }
}

__global__ void k_null(float *o) {
  if (threadIdx.x == 1023) o[1] = 0;
}

// host round trip of a blocking launch (launch + hipStreamSynchronize), the floor under a blocking exchange()
static void roundtrip(float *o, f4 *b, long n4) {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  auto run = [&](const char *name, auto launch) {
    for (int i = 0; i < 20; ++i) {
      launch();
      CK(hipStreamSynchronize(s));
    }
    const int reps = 200;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) {
      launch();
      CK(hipStreamSynchronize(s));
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
    auto t1 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) launch();
    CK(hipStreamSynchronize(s));
    const double us2 = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count() / reps;
    std::printf("roundtrip,%s,blocking_us,%.2f,stream_ordered_us,%.2f\n", name, us, us2);
    std::fflush(stdout);
  };
  run("null_kernel", [&] { k_null<<<1, 1024, 0, s>>>(o); });
  // 12.68 MB written (the 512^3 depth-2 self-exchange's payload) as one grid-stride store stream
  const long w4 = 12681216 / 16;
  run("write_12.7MB", [&] { k_write<false><<<1024, 256, 0, s>>>(b, w4, 1.f); });
  run("copy_12.7MB", [&] { k_copy<false><<<1024, 256, 0, s>>>(b + n4 / 2, b, w4); });
  CK(hipStreamDestroy(s));
}

int main(int argc, char **argv) {
  const int X = 512, Y = 512, Z = 512;
  const long n4 = long(X) * Y * Z / 4;
  const double bytes = double(n4) * 16;
  f4 *a, *b;
  float *o;
  CK(hipMalloc(&a, n4 * 16));
  CK(hipMalloc(&b, n4 * 16));
  CK(hipMalloc(&o, 64));
  CK(hipMemset(a, 0, n4 * 16));
  CK(hipMemset(b, 0, n4 * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time = [&](const char *name, int blocks, int waves, double mult, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    float best = 1e30f, sum = 0;
    const int reps = 10;
    for (int i = 0; i < reps; ++i) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
      sum += ms;
    }
    std::printf("%s,%d,%d,%.1f,%.3f,%.3f\n", name, blocks, waves, best * 1e3, mult * bytes / (best * 1e-3) / 1e12,
                mult * bytes / (sum / reps * 1e-3) / 1e12);
    std::fflush(stdout);
  };
  roundtrip(o, b, n4);
  if (argc > 1 && std::string(argv[1]) == "--roundtrip") return 0;
  std::printf("name,blocks,waves_per_block,best_us,best_TBps,mean_TBps\n");
  for (int blocks : {1024, 2048, 4096, 8192}) {
    time("copy", blocks, 4, 2, [&] { k_copy<false><<<blocks, 256>>>(a, b, n4); });
    time("copy_nt", blocks, 4, 2, [&] { k_copy<true><<<blocks, 256>>>(a, b, n4); });
    time("write", blocks, 4, 1, [&] { k_write<false><<<blocks, 256>>>(b, n4, 1.f); });
    time("write_nt", blocks, 4, 1, [&] { k_write<true><<<blocks, 256>>>(b, n4, 1.f); });
    time("read", blocks, 4, 1, [&] { k_read<<<blocks, 256>>>(a, n4, o); });
  }
#define ROWS(NW, PF, NT, NQ)                                                                                           \
  time("rows_nw" #NW "_pf" #PF "_nt" #NT "_q" #NQ, (Y / NW) * NQ, NW, 2,                                             \
       [&] { k_rows<NW, PF, NT><<<(Y / NW) * NQ, dim3(64, NW)>>>(a, b, Y, Z, NQ); })
  // 512 / 8 = 64 columns x 4 quarters = 256 blocks (the fused pair's 12-wave block has 8 output rows)
  ROWS(8, 1, true, 4);
  ROWS(8, 2, true, 4);
  ROWS(8, 3, true, 4);
  ROWS(8, 1, false, 4);
  ROWS(8, 3, false, 4);
  ROWS(16, 1, true, 4);
  ROWS(16, 3, true, 4);
  ROWS(16, 3, true, 8);
  ROWS(8, 3, true, 8);
  ROWS(4, 3, true, 4);
  ROWS(4, 3, true, 8);
  return 0;
}
