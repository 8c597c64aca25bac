// exhaustive: for every positive finite float s, the FMA-corrected quotient vs IEEE s / 6
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
int main() {
  const float c = 1.0f / 6.0f;
  uint32_t firstBad = 0, lastBad = 0, nbad = 0;
  for (uint32_t u = 1; u < 0x7f800000u; ++u) {
    float s;
    std::memcpy(&s, &u, 4);
    const float q0 = s * c;
    const float r = std::fmaf(-q0, 6.0f, s);
    const float q = std::fmaf(r, c, q0);
    const float ref = s / 6.0f;
    if (std::memcmp(&q, &ref, 4) != 0) {
      if (!nbad) firstBad = u;
      lastBad = u;
      ++nbad;
    }
  }
  float fb, lb;
  std::memcpy(&fb, &firstBad, 4);
  std::memcpy(&lb, &lastBad, 4);
  std::printf("mismatches %u, smallest %a, largest %a (log2 %.2f)\n", nbad, fb, lb, nbad ? std::log2(lb) : 0.0);
  return 0;
}
