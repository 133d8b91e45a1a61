// CPU exhaustive check of the FMA-corrected constant-divisor quotient (mm_models.h fast_quot_)
// against IEEE division for the C3 divisors, mismatches binned by input exponent:
//   gcc -O2 -ffp-contract=off tools/divchk.c -o /tmp/divchk -lm && /tmp/divchk   (~6 min)
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
static float asf(uint32_t u){float f; memcpy(&f,&u,4); return f;}
static uint32_t asu(float f){uint32_t u; memcpy(&u,&f,4); return u;}
int main(int argc, char** argv){
  float ds[5] = {6144.0f, 3072.0f, 6.28318548202514648f, 3.14159274101257324f, 0};
  ds[4] = (float)(1. / tan(M_PI / 3072));
  for (int k = 0; k < 5; k++) {
    volatile float d = ds[k]; float r = 1.0f / d;
    long bad[256] = {0}; long nb = 0;
    for (uint64_t u = 0; u < (1ull<<32); u++) {
      uint32_t b = (uint32_t)u; if (((b >> 23) & 0xff) == 0xff) continue;
      float x = asf(b);
      float q0 = x * r; float e = fmaf(-q0, d, x); float q = fmaf(e, r, q0);
      q = asf((asu(q) & 0x7fffffffu) | (asu(q0) & 0x80000000u));
      float ref = x / d;
      if (asu(q) != asu(ref)) { bad[(b >> 23) & 0xff]++; nb++; }
    }
    printf("d=%.9g r=%.9g mismatches %ld; by input exponent:", (double)d, (double)r, nb);
    for (int e = 0; e < 256; e++) if (bad[e]) printf(" [%d]=%ld", e - 127, bad[e]);
    printf("\n"); fflush(stdout);
  }
}
