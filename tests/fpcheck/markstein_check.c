/* tests/fpcheck/markstein_check.c — TEST-ONLY: checks that the quotient
 * sequence used by the kernel,
 *     y  = RN(1/b)            (correctly rounded reciprocal, once per ray)
 *     q0 = RN(a*y); r0 = fma(-q0,b,a); q1 = fma(r0,y,q0);
 *     r1 = fma(-q1,b,a);       q2 = fma(r1,y,q1)
 * returns RN(a/b) (Markstein's theorem: q1 is faithful, y is within half an
 * ulp of 1/b, so r1 is exact and q2 is the correctly rounded quotient), over
 * random and adversarial operands in the range the kernel admits
 * (2^-60 <= b <= 2^60, any a): the kernel only needs the quotient to decide
 * `u > 1e-5f && u < 10000.f` and, when that holds, its exact value; this
 * program checks exactly that property.
 * Built with -mfma so fmaf is the hardware fused multiply-add. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 0x9e3779b97f4a7c15ull;
static inline uint64_t nx(void) {
  uint64_t z = (s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
static inline float fbits(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline uint32_t ubits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static inline float mdiv(float a, float b, float y) {
  float q0 = a * y;
  float r0 = fmaf(-q0, b, a);
  float q1 = fmaf(r0, y, q0);
  float r1 = fmaf(-q1, b, a);
  return fmaf(r1, y, q1);
}

int main(int argc, char** argv) {
  long long N = argc > 1 ? atoll(argv[1]) : 200000000LL;
  long long bad = 0, tested = 0;
  for (long long i = 0; i < N; ++i) {
    uint64_t r = nx();
    float b, a;
    int mode = (int)(r & 7);
    if (mode < 4) {  /* typical kernel range: den = 2|d|^2 around 2, numerators +-1e-3..1e4 */
      b = fbits((uint32_t)(0x3f000000u + (uint32_t)((r >> 8) % 0x01800000u)));   /* [0.5, 4) */
      a = fbits((uint32_t)(0x3a000000u + (uint32_t)((r >> 32) % 0x0f000000u)));  /* ~5e-4 .. 3e5 */
      if (r & (1ull << 63)) a = -a;
    } else {  /* full admitted exponent range, random significands */
      int eb = (int)((r >> 8) % 121) - 60;
      int eq = (int)((r >> 16) % 201) - 100;
      b = ldexpf(1.0f + (float)((r >> 24) & 0x7fffff) * 0x1p-23f, eb);
      float q = ldexpf(1.0f + (float)((r >> 40) & 0x7fffff) * 0x1p-23f, eq);
      a = q * b;
      if (mode == 5) a = fbits(ubits(a) + 1u);
      if (mode == 6) a = fbits(ubits(a) - 1u);
      if (r & (1ull << 63)) a = -a;
    }
    if (mode == 7) { /* numerators near the acceptance thresholds */
      float th = (r & 2) ? 1.0e-5f : 10000.f;
      a = fbits(ubits(th * b) + (uint32_t)((r >> 20) & 3) - 1u);
    }
    float y = 1.0f / b;
    float want = a / b;
    float got = mdiv(a, b, y);
    ++tested;
    /* The kernel only uses a quotient through `u > 1e-5f && u < 10000.f` and,
     * when that holds, its exact value (raytracer.h:121-133). */
    int accW = (want > 1.0e-5f) && (want < 10000.f);
    int accG = (got > 1.0e-5f) && (got < 10000.f);
    if (accW != accG || (accW && ubits(got) != ubits(want))) {
      if (bad < 10) printf("MISMATCH a=%a b=%a want=%a got=%a\n", a, b, want, got);
      ++bad;
    }
  }
  printf("tested %lld mismatches %lld\n", tested, bad);
  return bad != 0;
}
