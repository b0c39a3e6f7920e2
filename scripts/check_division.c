/* Host check of the exact-division identities the HIP kernel relies on (walker_hip.hip fdiv_exact /
 * ddiv_exact / fdiv_count): float x/m == (float)((double)x * RN64(1/m)), Markstein's corrected double
 * quotient, and x / M for an integer M from a reciprocal within two ulps.
 * Usage: check_division [n]   (prints mismatch counts; all must be 0). */
#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include <stdint.h>
#include <string.h>
static uint64_t s=88172645463325252ull;
static inline uint64_t xr(){ s^=s<<13; s^=s>>7; s^=s<<17; return s; }
static float rf(){ // random float with random exponent in a physical range, random sign
  uint32_t u = (uint32_t)xr();
  int e = 127 + (int)(xr()%60) - 30;
  u = (u & 0x807fffffu) | ((uint32_t)e<<23);
  float f; memcpy(&f,&u,4); return f;
}
static double rd(){ uint64_t u=xr(); int e=1023+(int)(xr()%80)-40; u=(u&0x800fffffffffffffull)|((uint64_t)e<<52); double d; memcpy(&d,&u,8); return d; }
int main(int argc, char** argv){
  long bad1=0,bad2=0,bad3=0,n=argc>1?atol(argv[1]):200000000;
  for(long i=0;i<n;i++){
    // (1) f32 x / f32 m exact via double reciprocal
    float x=rf(), m=fabsf(rf());
    double ym = 1.0/(double)m;
    float q1 = (float)((double)x*ym);
    if (q1 != x/m) bad1++;
    // (2) double t / f32-valued double m, Markstein with y = RN(1/m)
    double t = rd(); double md=(double)m;
    double q = t*ym; double r = fma(-q, md, t); double q2 = fma(r, ym, q);
    if (q2 != t/md) bad2++;
    // (3) double (f32 value) / f32 cur (the spring t = fv/dist)
    double fv=(double)rf(); double c=(double)fabsf(rf()); double yc=1.0/c;
    double qq = fv*yc; double rr=fma(-qq,c,fv); double q3=fma(rr,yc,qq);
    if (q3 != fv/c) bad3++;
  }
  printf("n=%ld bad f32-via-f64=%ld markstein(t/m)=%ld markstein(fv/c)=%ld\n", n, bad1, bad2, bad3);
  // adversarial: m with all-ones mantissa, t near multiples
  long b4=0;
  for (long i=0;i<n/4;i++){
    uint32_t u = 0x3f800000u | (0x7fffffu - (uint32_t)(xr()%64)); float m; memcpy(&m,&u,4);
    double t = (double)(int64_t)(xr()>>11) * ldexp(1.0, -(int)(xr()%60));
    double ym=1.0/(double)m; double q=t*ym; double r=fma(-q,(double)m,t); double q2=fma(r,ym,q);
    if (q2 != t/(double)m) b4++;
    float x; uint32_t ux = (uint32_t)xr() & 0x7fffffffu; if (((ux>>23)&0xff)==0xff || ((ux>>23)&0xff)==0) continue; memcpy(&x,&ux,4);
    if ((float)((double)x*ym) != x/m) b4++;
  }
  printf("adversarial bad=%ld\n", b4);
  /* (5) fdiv_count: float x / M for an integer M < 2^11 as (float)(x * y), y within two ulps of 1/M (rcp64_nr),
   * |x| >= 2^-100: random x over the whole exponent range, and x = M * (a float rounding midpoint) nudged */
  long b5=0, n5=0;
  for (long i=0;i<n/4;i++){
    const int M = 1 + (int)(xr()%2047);
    const double y0 = 1.0/(double)M;
    const double ys[5] = {y0, nextafter(y0,0), nextafter(y0,1), nextafter(nextafter(y0,0),0), nextafter(nextafter(y0,1),1)};
    float x;
    if (i & 1) { uint32_t ux = (uint32_t)xr(); memcpy(&x,&ux,4); }
    else {
      const uint64_t k = (xr() & 0xffffffull) | 0x1000001ull;           /* 25-bit odd significand: a midpoint */
      const double mid = (double)k * ldexp(1.0, -(int)(xr()%200) + 60);
      x = (float)(mid * (double)M);
      const int nudge = (int)(xr()%5) - 2;
      for (int j=0;j<nudge;j++) x = nextafterf(x, INFINITY);
      for (int j=0;j>nudge;j--) x = nextafterf(x, -INFINITY);
      if (xr() & 1) x = -x;
    }
    if (!isfinite(x) || !(fabsf(x) >= 0x1p-100f)) continue;
    const float ref = x/(float)M;
    n5++;
    for (int j=0;j<5;j++) if ((float)((double)x*ys[j]) != ref) b5++;
  }
  printf("count-divisor n=%ld bad=%ld\n", n5, b5);
  /* (6) the float32 quotients' exact range (walker_hip.hip TINY_EXP / divisor_ok): dividend 0 or |x| >= 2^-80, divisor
   * |m| in [2^-20, 2^21), finite quotient: Markstein's float32 step from RN32(1/m), the double product with RN64(1/m)
   * (fdiv_exact) and with a reciprocal two ulps off (fdiv_rcp from rcp64_nr) all equal IEEE x / m.  Dividends drawn
   * over the whole range and concentrated near its low end, divisors near the range's ends too. */
  long b6=0, n6=0;
  for (long i=0;i<n/2;i++){
    uint32_t ux=(uint32_t)xr(); int ex = (i & 1) ? 127-80+(int)(xr()%208) : 127-80+(int)(xr()%24);
    if (ex > 254) continue;
    ux=(ux&0x807fffffu)|((uint32_t)ex<<23); float x; memcpy(&x,&ux,4);
    if (xr()%64==0) x = 0.0f;
    uint32_t um=(uint32_t)xr(); int em = (i & 2) ? 127-20+(int)(xr()%41) : ((i & 4) ? 127-20+(int)(xr()%3) : 127+18+(int)(xr()%3));
    um=(um&0x007fffffu)|((uint32_t)em<<23); float m; memcpy(&m,&um,4);
    if (xr()&1) m = -m;
    const float ref = x/m;
    if (!isfinite(ref)) continue;
    n6++;
    const float yf = (float)(1.0/(double)m);
    const float q = x*yf, r = fmaf(-q, m, x), qm = fmaf(r, yf, q);
    if (memcmp(&qm,&ref,4)) b6++;
    const double y0 = 1.0/(double)m;
    const double ys[3] = {y0, nextafter(nextafter(y0,0),0), nextafter(nextafter(y0,INFINITY),INFINITY)};
    for (int j=0;j<3;j++){ const float qd=(float)((double)x*ys[j]); if (memcmp(&qd,&ref,4)) b6++; }
  }
  printf("exact-range n=%ld bad=%ld\n", n6, b6);
  return (bad1||bad2||bad3||b4||b5||b6) ? 1 : 0;
}
