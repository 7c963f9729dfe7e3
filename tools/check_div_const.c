/* Exhaustive check behind ipt_device.h::div_const: for the constant divisors
 * b of the hot path (1/pi as a float, 0.9, pi as a float), with y = RN(1/b),
 *     q = RN(x * y);  r = fma(-q, b, x);  RN(fma(r, y, q)) == RN(x / b)
 * for EVERY float 2^-100 <= x < 2^100 (negative x follows by symmetry: every
 * step is odd in x under round-to-nearest-even).  Host IEEE: divss, fmaf
 * (-mfma: the hardware fused multiply-add).  Prints the mismatch count per
 * constant; exit status 1 if any.
 *     gcc -O2 -mfma -fopenmp tools/check_div_const.c -o /tmp/check_div_const */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t u_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

int main(void) {
  const float consts[3] = {(float)(1.0 / 3.14159265358979323846), 0.9f, (float)3.14159265358979323846};
  const char *names[3] = {"1/pi", "0.9", "pi"};
  const uint32_t lo = u_of(0x1p-100f), hi = u_of(0x1p100f);
  int bad_any = 0;
  for (int c = 0; c < 3; ++c) {
    const float b = consts[c];
    const float y = (float)(1.0 / (double)b);
    volatile float bv = b;  /* keep the IEEE division a real division */
    long long bad = 0;
#pragma omp parallel for reduction(+ : bad) schedule(static)
    for (int64_t i = lo; i < (int64_t)hi; ++i) {
      const float x = f_of((uint32_t)i);
      const float q = x * y;
      const float r = fmaf(-q, b, x);
      const float z = fmaf(r, y, q);
      const float w = x / bv;
      if (u_of(z) != u_of(w)) ++bad;
    }
    printf("b = %s (%a), y = %a: %lld mismatches over [2^-100, 2^100)\n", names[c], b, y, bad);
    bad_any |= bad != 0;
  }
  return bad_any;
}
