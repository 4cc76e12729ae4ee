// Host check of the catch-up Adam's division by a per-step constant
// (csrc/optim.hip adam_zero_step): for d = bc2_sqrt of step t and its
// correctly rounded reciprocal r = RN(1/d), q0 = RN(x·r), e = fma(−q0, d, x),
// q = fma(e, r, q0) must equal RN(x / d) (Markstein's theorem: r within ½ ulp
// of 1/d, q0 within 1 ulp of x/d, no underflow in e — x here is sqrt(v) ≥ 2^-75).
// Every mantissa of x at several exponents for the first steps' d, random x for
// the rest.  gcc -O2 -ffp-contract=off tools/markstein_check.c -lm
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float bits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

static long check(float x, float d, float r) {
  const float q0 = x * r;
  const float e = fmaf(-q0, d, x);
  const float q = fmaf(e, r, q0);
  const float ref = x / d;
  return memcmp(&q, &ref, 4) != 0;
}

int main(void) {
  const float betas[] = {0.999f, 0.99f, 0.98f, 0.9f};
  long bad = 0, n = 0;
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (int bi = 0; bi < 4; ++bi) {
    const float b2 = betas[bi];
    for (int t = 1; t <= 20000; ++t) {
      // bc2_sqrt as the host computes it: sqrt(1 - beta2^t) in fp32
      const float bc2 = sqrtf(1.0f - powf(b2, (float)t));
      if (!(bc2 > 0.f)) continue;
      const float r = 1.0f / bc2;
      const int exhaustive = (bi == 0 && (t <= 4 || t % 997 == 0));
      if (exhaustive) {
        for (int ex = -75; ex <= 20; ex += 19)
          for (uint32_t m = 0; m < (1u << 23); ++m) {
            bad += check(bits(((uint32_t)(ex + 127) << 23) | m), bc2, r);
            ++n;
          }
      } else {
        for (int k = 0; k < 4096; ++k) {
          s ^= s << 13; s ^= s >> 7; s ^= s << 17;
          const int ex = -75 + (int)((s >> 40) % 96);
          const uint32_t m = (uint32_t)(s & 0x7FFFFF);
          bad += check(bits(((uint32_t)(ex + 127) << 23) | m), bc2, r);
          ++n;
        }
      }
    }
  }
  bad += check(0.f, 0.5f, 2.0f);
  printf("markstein: %ld of %ld quotients differ from x / d\n", bad, n);
  return bad != 0;
}
