// CPU check of the fp64 exact-division-by-6 sequence used in the stencil kernels (g++ -O2 -o div6 div6_fp64_check.cpp -lpthread)
// randomized check: q = fma(fma(-x*c, 6, x), c, x*c) == x / 6 for doubles with |x| >= 2^-960
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>
#include <atomic>
int main() {
  const double c = 1.0 / 6.0;
  std::atomic<long> bad{0}, n{0};
  auto work = [&](int tid) {
    std::mt19937_64 g(1234 + tid);
    long lb = 0, ln = 0;
    for (long i = 0; i < 150000000L; ++i) {
      uint64_t b = g();
      // exponent restricted to [2^-960, 2^1023]; also bias toward mantissas near multiples of 3 (hard cases)
      uint64_t e = 63 + (b >> 52) % (2046 - 63);
      uint64_t m = b & ((1ULL << 52) - 1);
      if ((i & 3) == 0) m = (m / 3) * 3 + (i & 4 ? 1 : 2) % 3;
      uint64_t bits = (b & (1ULL << 63)) | (e << 52) | (m & ((1ULL << 52) - 1));
      double x;
      std::memcpy(&x, &bits, 8);
      if (std::fabs(x) < 0x1p-960) continue;
      const double q0 = x * c;
      const double r = std::fma(-q0, 6.0, x);
      const double q = std::fma(r, c, q0);
      const double t = x / 6.0;
      ++ln;
      if (std::memcmp(&q, &t, 8) != 0) {
        if (lb < 5) std::printf("mismatch x=%a q=%a t=%a\n", x, q, t);
        ++lb;
      }
    }
    bad += lb;
    n += ln;
  };
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t) th.emplace_back(work, t);
  for (auto &t : th) t.join();
  std::printf("checked %ld, mismatches %ld\n", n.load(), bad.load());
}
