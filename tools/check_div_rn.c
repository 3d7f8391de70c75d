/* Brute-force check that div_rn (csrc/unproject.hip) equals IEEE a / b:
 * gcc -O2 -ffp-contract=off tools/check_div_rn.c -lm -o /tmp/check_div_rn && /tmp/check_div_rn 200000000 */
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
static uint64_t s = 88172645463325252ull;
static inline uint64_t xr(void){ s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static inline double rnd_sig(int e0, int e1){ uint64_t m = xr() & ((1ull<<52)-1); int e = e0 + (int)(xr() % (uint64_t)(e1-e0+1)); uint64_t bits = ((uint64_t)(e+1023) << 52) | m; double d; memcpy(&d,&bits,8); return d; }
int main(int argc, char** argv){
  long n = atol(argv[1]); long bad = 0;
  for (long i = 0; i < n; ++i) {
    double b = rnd_sig(-3, 12);
    if (i % 7 == 0) { uint64_t bits; memcpy(&bits,&b,8); bits |= ((1ull<<52)-1) - (xr()&15); memcpy(&b,&bits,8); }
    double a = rnd_sig(-30, 14) * ((xr()&1) ? 1 : -1);
    double r = 1.0 / b;
    double q0 = a * r;
    double rem = fma(-q0, b, a);
    double q = fma(rem, r, q0);
    double e = a / b;
    if (q != e) { if (bad < 10) printf("a=%.17g b=%.17g q=%.17g e=%.17g\n", a, b, q, e); ++bad; }
  }
  printf("bad %ld of %ld\n", bad, n);
}
