// Check of div_const (csrc/dpft_ic.hip, make_taps_xy's division by the level's constant
// (W - 1) / 2 and (H - 1) / 2): for divisor b, y = RN(1/b), q0 = RN(a*y), r = fma(-q0,b,a),
// q1 = fma(r,y,q0) must equal RN(a/b) for every float a the kernel divides (|a| <= 2^30; quotients
// below 2^-25 cannot move a tap, since (q - 1) + 1 rounds to 0 for them either way).
//   gcc -O3 -ffp-contract=off -o /tmp/div_check tools/div_check.c -lm
//   /tmp/div_check 0      all 2^32 floats for the twelve verified divisors (~14 min): every level of
//                         640x480 and 160x120 (W, H = 640 .. 20, 480 .. 15) -- the set the library
//                         selects div_const for (kVerifiedTapSizes in csrc/dpft_ic.hip); any other
//                         size takes the IEEE division
//   /tmp/div_check 3      all 2^32 floats for the four sizes below 80 x 60 only (~5 min)
//   /tmp/div_check 1      every size n = 2..8192, a stride of 4099 through all floats (~3 min)
//   /tmp/div_check 2      quick: the eight divisors, a stride of 65537 (tests/test_div_check.py)
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <stdlib.h>
static inline float f_of(uint32_t u){float f; memcpy(&f,&u,4); return f;}
static inline uint32_t u_of(float f){uint32_t u; memcpy(&u,&f,4); return u;}
long check(float b, uint64_t lo, uint64_t hi, uint64_t step) {
  volatile float bv = b;
  const float y = 1.0f / bv;
  long bad = 0;
  for (uint64_t i = lo; i < hi; i += step) {
    const float a = f_of((uint32_t)i);
    if (!isfinite(a) || fabsf(a) > 1073741824.0f) continue;  // |u| > 2^30: clamped before the division
    const float q = a / b;
    const float q0 = a * y;
    const float r = fmaf(-q0, b, a);
    const float q1 = fmaf(r, y, q0);
    if (fabsf(q) < 2.9802322e-08f && fabsf(q1) < 2.9802322e-08f) continue;  // |q| < 2^-25: (q - 1) + 1 == 0 either way
    if (u_of(q) != u_of(q1)) {
      if (bad < 5) printf("  mismatch b=%.9g a=%.9g (%08x): div %.9g (%08x) seq %.9g (%08x)\n", b, a, (uint32_t)i, q, u_of(q), q1, u_of(q1));
      ++bad;
    }
  }
  return bad;
}
int main(int argc, char** argv) {
  int mode = atoi(argv[1]);
  if (mode == 0 || mode == 3) {  // exhaustive for the verified divisors
    float ds[] = {319.5f, 159.5f, 79.5f, 39.5f, 239.5f, 119.5f, 59.5f, 29.5f, 19.5f, 9.5f, 14.5f, 7.0f};
    long tot = 0;
    for (int k = mode == 3 ? 8 : 0; k < 12; ++k) {
      long bad = check(ds[k], 0, 1ull<<32, 1); tot += bad; printf("b=%g bad=%ld\n", ds[k], bad); fflush(stdout);
    }
    printf("exhaustive: total bad %ld\n", tot);
    return tot != 0;
  } else if (mode == 2) {  // quick
    float ds[] = {319.5f, 159.5f, 79.5f, 39.5f, 239.5f, 119.5f, 59.5f, 29.5f};
    long tot = 0;
    for (int k = 0; k < 8; ++k) tot += check(ds[k], 0, 1ull<<32, 65537);
    printf("quick: total bad %ld\n", tot);
    return tot != 0;
  } else {  // every size n = 2..8192 (b = (n-1)/2), strided a
    long tot = 0;
    for (int n = 2; n <= 8192; ++n) { float b = (float)(n - 1) * 0.5f; long bad = check(b, 0, 1ull<<32, 4099); tot += bad; if (bad) printf("n=%d bad=%ld\n", n, bad);}
    printf("sizes 2..8192 strided: total bad %ld\n", tot);
  }
}
