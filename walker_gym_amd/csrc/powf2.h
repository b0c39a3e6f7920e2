/* powf2.h — numpy's float32 `x ** 2`, bit for bit, for the kernel (HIP device code) and the host checks (C).
 *
 * numpy evaluates `np.float32 ** 2` (a scalar power: `np.linalg.norm(p.v) ** 2` in PhysicsEnv._calculate_energy,
 * gym/optimized_env.py:242; `distance ** 2` in Point.gravity_vec, gym/optimized_engine.py:185-189) with libm
 * powf, and glibc's powf is NOT x*x: it is exp2(y * log2(x)) evaluated in double and rounded once, within 0.82 ulp
 * (e.g. powf(673.88745f, 2) = 454124.3125f where x*x = 454124.28125f; ~0.07% of random inputs differ).  This file
 * restates that published algorithm (glibc 2.35 sysdeps/ieee754/flt-32/e_powf.c, the ARM optimized-routines powf:
 * a 16-entry log2 table with an order-5 polynomial, a 32-entry exp2 table with an order-3 polynomial) at y = 2,
 * with glibc's own table and polynomial constants (__powf_log2_data, __exp2f_data).  Pinned exhaustively: every
 * non-negative finite float32 gives libm's bits (scripts/check_powf2.c, tests/test_powf2.py; the fused and the
 * unfused evaluation of the polynomials both match).
 *
 * pw_pow2(x) is the full evaluation.  pw_pow2_fast(x, &f) returns 1 and f = RN(x*x) when that provably equals it:
 * the double pre-rounding value of the algorithm lies within ~1.65e-3 ulp of x^2 for every float (measured over all
 * of them), so when x^2 +- 1.75e-3 ulp round to the same float, so does the algorithm's value.
 */
#ifndef WALKER_POWF2_H
#define WALKER_POWF2_H

#if defined(__HIPCC__) || defined(__HIP__)
#define PW_FN __device__ __forceinline__
#define PW_TAB static __constant__
#define PW_FMA(a, b, c) __builtin_fma((a), (b), (c))
#else
#include <math.h>
#include <stdint.h>
#include <string.h>
#define PW_FN static inline
#define PW_TAB static const
#define PW_FMA(a, b, c) fma((a), (b), (c))
#endif

/* __powf_log2_data.tab: {invc, logc} of 16 subintervals of [0x3f330000, 2 * 0x3f330000) (POWF_SCALE = 1) */
PW_TAB double PW_LOG2_TAB[32] = {
    0x1.661ec79f8f3bep+0, -0x1.efec65b963019p-2, 0x1.571ed4aaf883dp+0, -0x1.b0b6832d4fca4p-2,
    0x1.49539f0f010b0p+0, -0x1.7418b0a1fb77bp-2, 0x1.3c995b0b80385p+0, -0x1.39de91a6dcf7bp-2,
    0x1.30d190c8864a5p+0, -0x1.01d9bf3f2b631p-2, 0x1.25e227b0b8ea0p+0, -0x1.97c1d1b3b7af0p-3,
    0x1.1bb4a4a1a343fp+0, -0x1.2f9e393af3c9fp-3, 0x1.12358f08ae5bap+0, -0x1.960cbbf788d5cp-4,
    0x1.0953f419900a7p+0, -0x1.a6f9db6475fcep-5, 0x1.0000000000000p+0, 0x0.0p+0,
    0x1.e608cfd9a47acp-1, 0x1.338ca9f24f53dp-4, 0x1.ca4b31f026aa0p-1, 0x1.476a9543891bap-3,
    0x1.b2036576afce6p-1, 0x1.e840b4ac4e4d2p-3, 0x1.9c2d163a1aa2dp-1, 0x1.40645f0c6651cp-2,
    0x1.886e6037841edp-1, 0x1.88e9c2c1b9ff8p-2, 0x1.767dcf5534862p-1, 0x1.ce0a44eb17bccp-2};
/* __exp2f_data.tab: bits of RN(2^(i/32)) minus i << 47 */
PW_TAB unsigned long long PW_EXP2_TAB[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};

PW_FN double pw_asdouble(unsigned long long u) {
    double d;
#if defined(__HIPCC__) || defined(__HIP__)
    d = __builtin_bit_cast(double, u);
#else
    memcpy(&d, &u, 8);
#endif
    return d;
}
PW_FN unsigned long long pw_asu64(double d) {
    unsigned long long u;
#if defined(__HIPCC__) || defined(__HIP__)
    u = __builtin_bit_cast(unsigned long long, d);
#else
    memcpy(&u, &d, 8);
#endif
    return u;
}
PW_FN unsigned int pw_asu32(float f) {
    unsigned int u;
#if defined(__HIPCC__) || defined(__HIP__)
    u = __builtin_bit_cast(unsigned int, f);
#else
    memcpy(&u, &f, 4);
#endif
    return u;
}
PW_FN float pw_asfloat(unsigned int u) {
    float f;
#if defined(__HIPCC__) || defined(__HIP__)
    f = __builtin_bit_cast(float, u);
#else
    memcpy(&f, &u, 4);
#endif
    return f;
}

/* glibc powf(x, 2.0f): log2_inline, y * log2(x) (exact doubling), exp2_inline, one rounding to float */
PW_FN float pw_pow2(float x) {
    unsigned int ix = pw_asu32(x) & 0x7fffffffu;   /* y = 2 is an even integer: no sign bias */
    if (ix == 0u || ix >= 0x7f800000u) return x * x;   /* zero, inf, nan: glibc returns x * x */
    if (ix < 0x00800000u) {                           /* subnormal: normalise (the product is exact) */
        ix = pw_asu32(pw_asfloat(ix) * 0x1p23f) & 0x7fffffffu;
        ix -= 23u << 23;
    }
    const unsigned int tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) & 15u);
    const unsigned int top = tmp & 0xff800000u;
    const int k = (int)top >> 23;
    const double invc = PW_LOG2_TAB[2 * i], logc = PW_LOG2_TAB[2 * i + 1];
    const double z = (double)pw_asfloat(ix - top);
    const double r = PW_FMA(z, invc, -1.0);
    const double y0 = logc + (double)k;
    const double r2 = r * r;
    double y = PW_FMA(0x1.27616c9496e0bp-2, r, -0x1.71969a075c67ap-2);
    const double p = PW_FMA(0x1.ec70a6ca7baddp-2, r, -0x1.7154748bef6c8p-1);
    const double r4 = r2 * r2;
    double q = PW_FMA(0x1.71547652ab82bp+0, r, y0);
    q = PW_FMA(p, r2, q);
    y = PW_FMA(y, r4, q);
    const double xd = 2.0 * y;
    if (((pw_asu64(xd) >> 47) & 0xffffu) >= (pw_asu64(126.0) >> 47)) {   /* |2 log2 x| >= 126 */
        if (xd > 0x1.fffffffd1d571p+6) return pw_asfloat(0x7f800000u);   /* overflow: +inf */
        if (xd <= -150.0) return 0.0f;                                    /* underflow: +0 */
    }
    const double shift = 0x1.8p+47;   /* 0x1.8p+52 / 32 */
    double kd = xd + shift;
    const unsigned long long ki = pw_asu64(kd);
    kd -= shift;
    const double rr = xd - kd;
    const unsigned long long t = PW_EXP2_TAB[ki & 31u] + (ki << 47);
    const double s = pw_asdouble(t);
    const double zz = PW_FMA(0x1.c6af84b912394p-5, rr, 0x1.ebfce50fac4f3p-3);
    const double rr2 = rr * rr;
    double yy = PW_FMA(0x1.62e42ff0c52d6p-1, rr, 1.0);
    yy = PW_FMA(zz, rr2, yy);
    return (float)(yy * s);
}

/* RN(x*x) when it provably equals pw_pow2(x) (returns 1), else 0 (call pw_pow2).  Finite x only.
 * The band: PW_FAST_C ulps of e's float binade (2^(E-24) for e = m 2^E, m in [0.5, 1)); e = 0 is exact.  1.75e-3 ulps
 * sits just above the algorithm's largest deviation (the exhaustive sweep passes at 1.68e-3 and fails 1,274 inputs at
 * 1.60e-3, profiles/r04_powf2_band.json) and sends 0.180 % of all floats to pw_pow2, against 0.293 % for the earlier
 * relative band 2^-32 e (1.95e-3 to 3.9e-3 ulps across a binade; PW_FAST_C = 0 restores it). */
#ifndef PW_FAST_C
#define PW_FAST_C 1.75e-3
#endif
PW_FN int pw_pow2_fast(float x, float *out) {
    const double e = (double)x * (double)x;          /* exact: 48 significant bits */
    double d;
    if (PW_FAST_C > 0.0) {
#if defined(__HIPCC__) || defined(__HIP__)
        d = __builtin_amdgcn_ldexp(PW_FAST_C, __builtin_amdgcn_frexp_exp(e) - 24);
#else
        int E;
        (void)frexp(e, &E);
        d = ldexp(PW_FAST_C, E - 24);
#endif
    } else {
        d = e * 0x1p-32;
    }
    const float lo = (float)(e - d), hi = (float)(e + d);
    *out = (float)e;
    return lo == hi || e == 0.0;
}

#endif /* WALKER_POWF2_H */
