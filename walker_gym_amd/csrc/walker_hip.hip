// walker_hip.hip — MI355X (gfx950 / CDNA4) batched walker stepper + the C ABI of include/walker_hip.h.
//
// One launch = one env step for every walker:
//   act (Muscle.act/regulation)  ->  springs in edge order  ->  gravity, damp, ground  ->
//   symplectic Euler (Point.run1)  ->  observation, reward, done, info.
//
// Execution model:
//   * a workgroup owns a CONTIGUOUS range of walkers, so every SoA array it touches is one contiguous
//     byte range in HBM.  Phase 0 issues EVERY global load of the tile back to back (state -> LDS with
//     16-B loads; edge / muscle / incidence-offset records -> registers of the lane that uses them),
//     so the tile pays one HBM latency, not a chain of them;
//   * act: muscle lanes update the rest lengths straight from registers;
//   * edge phase: one lane per edge computes the spring term t = RN64(f*dir / dist) and the damping
//     force df (float32) ONCE, into LDS;
//   * mass phase: one lane per mass walks its incidence list (LDS, sorted by edge index) and
//     accumulates a = f32(f64(a) + t/m) then a += df/m in exactly the reference's order, then env
//     forces and the integrator in registers — deterministic, no atomics;
//   * observe: per-walker reductions in numpy's summation order (8 lanes per walker), obs rows written
//     as one contiguous coalesced block.
// Compiled with -ffp-contract=off and IEEE f32/f64 division/sqrt (build.py), so each float op rounds
// exactly as numpy's does.

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "walker_hip.h"
#include "powf2.h"

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

constexpr int WG_MAX_M = 1024;      // numpy pairwise recursion unrolled 3 levels (pw_tree<3>)
constexpr double CONFIG_R = 16e-36;  // gym/engine.py:9 Config.r (distance clamp, Python float)
constexpr int EPL = 4;               // edges per lane per pass held in registers
constexpr int NTHREADS = 256;           // default workgroup size (walkers fill 256 mass lanes)
constexpr int MAXT = 512;               // __launch_bounds__: workgroups are 64..512 threads (> 256: M > 64 only)
// Diagnostic builds only (scripts/variant_ab.py, -DWG_ABLATE=bits): bit k skips phase k of the step to price it.  Such a
// build's results are NOT exact (tests/test_abi.py compiles one; no GPU test loads it); 0 in the product.
#ifndef WG_ABLATE
#define WG_ABLATE 0
#endif

// Float32 constants derived from wg_params exactly where numpy rounds the Python scalars.
struct KParams {
    float neg_g, neg_dampk, ground, neg_groundk, neg_grounddamp, friction, dt;
    float pk, vk, ak, mk, done_y;
    float dt2;      // run2: float32(t ** 2), t**2 a Python float (double) cast where numpy casts it
    double g;
    int max_steps, midform, conmid, spring_mode, action_mode;
    int integrator; // 2: Point.run2, otherwise Point.run1
    int pair_mode;  // bitmask, after the springs in bit order: 1 Point.gravity, 2 Point.coulomb, 4 Point.bounce,
                    // 8 G2 Point.gravity (gravity_vec: zero a, float32 pairs), 16 Point.electrostatic (every point)
    double pair_g, pair_k, pair_e;
    float bounce_kh;  // float32(k / 2) of Point.bounce(k)
    // spring_mode 2, the G3 engine (gym/optimized_walker/env.py:135-184), everything rounded to float32
    float g3g[3], g3_damp, g3_dragc, g3_level, g3_rest, g3_fric;   // g3_dragc = f32(-0.5 * air_resistance)
    int g3_ground;
    int friction_mode;   // 0: (-v)*(|deep|*friction) (gym/optimized_env.py:168-172); 1: (v*deep)*friction (gym/env.py:41)
    int prio;         // WG_LEAN_PRIO: 1 (default) raise the wave priority while a lean tile issues its loads, so a
                      // wave's HBM requests leave before other waves' arithmetic; 0 off
    int xcd;          // WG_XCD bitmask: XCD-aware workgroup order (xcd_block) for 1 the wave kernel, 2 the lean kernel
};

// The per-step outputs the step kernels write: wg_outputs without the opt-in info pointers (walker_info_kernel writes
// those), passed by value as a kernel argument.  (wg_outputs itself by value put its ABI-10 fields among the lean
// kernel's arguments: 20 more SGPR spill instructions, v_writelane / v_readlane, and +16 VALU per wave.)
struct KOut {
    float *obs, *reward;
    uint8_t *done;
    float *centroid, *energy;
    int32_t *steps;
    int64_t obs_step, out_step;
    int32_t obs_stride, obs_pad_clean;
};
inline KOut kout(const wg_outputs &o) {
    return KOut{o.obs, o.reward, o.done, o.centroid, o.energy, o.steps, o.obs_step, o.out_step, o.obs_stride,
                o.obs_pad_clean};
}

// Step-kernel launches.  wg_time_step (ABI 14, a measurement aid) sets the two events on this thread around each step it
// issues: the launch then goes through hipExtLaunchKernel, which stamps the kernel's own start and end on them (the
// dispatch's timestamps, as a kernel trace reports them); otherwise a plain launch.
thread_local hipEvent_t g_kev_start = nullptr, g_kev_stop = nullptr;
#define WG_KLAUNCH(KERNEL, GRID, BLOCK, LDS, STREAM, ...)                                                          \
    do {                                                                                                          \
        if (g_kev_start)                                                                                          \
            hipExtLaunchKernelGGL(KERNEL, GRID, BLOCK, LDS, STREAM, g_kev_start, g_kev_stop, 0u, __VA_ARGS__);    \
        else                                                                                                      \
            hipLaunchKernelGGL(KERNEL, GRID, BLOCK, LDS, STREAM, __VA_ARGS__);                                    \
    } while (0)

// XCD-aware workgroup order: MI355X deals workgroups round-robin over its 8 XCDs (each with its own L2; observed
// placement, speed only), so hardware block b runs on XCD group b % 8.  The guide's bijective T1 swizzle maps b to a
// logical block so that each XCD group takes one contiguous run of logical blocks, in launch order: consecutive
// tiles then share an L2 (their partial output lines merge there and their shared input lines are fetched once).
__device__ __forceinline__ int xcd_block(int bid, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

// Per-launch geometry: caps of one workgroup's slice (LDS carve sizes).
struct Geo {
    int W, Pcap, Ecap, Ucap;   // walkers, masses, edges, muscles per workgroup (max)
    int threads;
    int lds;
    float invM, invK, invA;    // uniform batches: 1/M, 1/K, 1/A for exact small-int division (fdiv)
    int tbytes;                // spring-term region, also the obs tile of uniform batches (aliased)
    int lite;                  // register-reduction kernels: no LDS for acc, m, reduction terms, offsets
};

// Diagnostic builds only (-DWG_STAMPS, scripts/stamps.py): lane 0 of every lean wave records s_memtime at its
// phase boundaries into g_stamps[wave][8] with a vector store; wg_debug_stamps copies them out.  Never in the
// product build.
#ifdef WG_STAMPS
__device__ unsigned long long g_stamps[(1 << 16) * 8];
#define STAMP(k)                                                                                          \
    do {                                                                                                  \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                      \
        if ((threadIdx.x & 63) == 0 && stamp_wave < (1 << 16)) g_stamps[stamp_wave * 8 + (k)] = t_;      \
    } while (0)
#else
#define STAMP(k) do {} while (0)
#endif

struct Carve {
    double *t;                   // [Ecap*3] spring term RN64(f*dir/dist)
    float *pos, *vel, *acc, *m;  // [Pcap*3] / [Pcap]
    float *df;                   // [Ecap*3] damping force
    uint32_t *inc;               // [Ecap]   incidence entries, two u16 per word
    float *x;                    // [Ucap]   muscle rest length after act
    float *nrm, *ke, *pe;        // [Pcap]   per-mass reduction terms
    float *red;                  // [W*8]    per-walker reductions
    int *moff, *eoff, *uoff;     // [W+1]    block-local walker offsets (ragged)
};

__host__ __device__ inline int align16(int b) { return (b + 15) & ~15; }

// the caller's index of stored walker w (its action row and output row; wg_batch.row, NULL = identity)
__device__ __forceinline__ int caller_row(const wg_batch &b, int w) { return b.row ? b.row[w] : w; }

// one carve for host sizing and device pointers.  The walk produces byte OFFSETS only; the device
// pointers are `smem + offset` with no null test in between, so the compiler keeps them in the LDS
// address space (a `base ? base + b : nullptr` select made them generic: flat loads/stores and the
// 15 pointers spilled to scratch in the ragged kernel).
enum { CV_T, CV_POS, CV_VEL, CV_ACC, CV_M, CV_DF, CV_INC, CV_X, CV_NRM, CV_KE, CV_PE, CV_RED,
       CV_MOFF, CV_EOFF, CV_UOFF, CV_N };
__host__ __device__ inline int carve_walk(const Geo &g, int *off) {
    int b = 0, k = 0;
    auto take = [&](int bytes) { off[k++] = b; b += align16(bytes); };
    const int full = g.lite ? 0 : 1;
    take(g.tbytes); take(g.Pcap * 12); take(g.Pcap * 12);                  // t, pos, vel
    take(full * g.Pcap * 12); take(full * g.Pcap * 4);                      // acc, m
    take(g.Ecap * 12);                                                      // df
    take(g.Ecap * 4 + 16); take(g.Ucap * 4);                                // inc, x
    take(full * g.Pcap * 4); take(full * g.Pcap * 4); take(full * g.Pcap * 4);   // nrm, ke, pe
    take(full * g.W * 32);                                                  // red
    take(full * (g.W + 1) * 4); take(full * (g.W + 1) * 4); take(full * (g.W + 1) * 4);   // moff, eoff, uoff
    return b;
}
__host__ __device__ inline int carve_bytes(const Geo &g) { int off[CV_N]; return carve_walk(g, off); }
__device__ inline Carve carve(char *s, const Geo &g) {
    int o[CV_N];
    carve_walk(g, o);
    Carve c;
    c.t = reinterpret_cast<double *>(s + o[CV_T]); c.pos = reinterpret_cast<float *>(s + o[CV_POS]);
    c.vel = reinterpret_cast<float *>(s + o[CV_VEL]); c.acc = reinterpret_cast<float *>(s + o[CV_ACC]);
    c.m = reinterpret_cast<float *>(s + o[CV_M]); c.df = reinterpret_cast<float *>(s + o[CV_DF]);
    c.inc = reinterpret_cast<uint32_t *>(s + o[CV_INC]); c.x = reinterpret_cast<float *>(s + o[CV_X]);
    c.nrm = reinterpret_cast<float *>(s + o[CV_NRM]); c.ke = reinterpret_cast<float *>(s + o[CV_KE]);
    c.pe = reinterpret_cast<float *>(s + o[CV_PE]); c.red = reinterpret_cast<float *>(s + o[CV_RED]);
    c.moff = reinterpret_cast<int *>(s + o[CV_MOFF]); c.eoff = reinterpret_cast<int *>(s + o[CV_EOFF]);
    c.uoff = reinterpret_cast<int *>(s + o[CV_UOFF]);
    return c;
}

// ------------------------------------------------------------------ numpy-exact float helpers
// np.linalg.norm of a float32 3-vector: OpenBLAS sdot (float products summed in double), float sqrt.
// sqrtf of a float s in [2^-96, 2^126): v_sqrt_f32 and the one-ulp correction, the same steps as the compiler's
// correctly rounded sqrtf minus its small-input rescaling and zero/inf fix-up, which this range never needs
__device__ __forceinline__ float sqrt_mid(float s) {
    const float r = __builtin_amdgcn_sqrtf(s);
    const float rd = __uint_as_float(__float_as_uint(r) - 1u), ru = __uint_as_float(__float_as_uint(r) + 1u);
    float o = (__builtin_fmaf(-rd, r, s) <= 0.f) ? rd : r;
    return (__builtin_fmaf(-ru, r, s) > 0.f) ? ru : o;
}
__device__ inline float np_norm3(float x, float y, float z) {
    const float px = x * x, py = y * y, pz = z * z;
    double s = 0.0;
    s += (double)px; s += (double)py; s += (double)pz;
    // (sqrt_mid where its range allows, the compiler's sqrtf elsewhere, ran 1 % slower: the branch costs more than
    // the rescaling it skips, profiles/r03zm_ab_norm_*.txt)
    return sqrtf((float)s);
}
__device__ inline float np_dot3(float ax, float ay, float az, float bx, float by, float bz) {
    const float p0 = ax * bx, p1 = ay * by, p2 = az * bz;
    double s = 0.0;
    s += (double)p0; s += (double)p1; s += (double)p2;
    return (float)s;
}
// numpy float32 pairwise summation (the add.reduce inner loop behind np.mean / np.sum) over a
// strided LDS array: < 8 sequential; <= 128 eight interleaved partial sums; above that numpy
// recurses on halves split at a multiple of 8.
// r + a[0] + a[st] + ... (n terms) left to right, the reads issued four at a time ahead of their adds (one LDS
// round trip per four terms instead of one per term; the same additions in the same order)
__device__ inline float seq_sum_lds(float r, const float *a, int n, int st) {
    int i = 0;
    for (; i + 4 <= n; i += 4) {
        const float x0 = a[i * st], x1 = a[(i + 1) * st], x2 = a[(i + 2) * st], x3 = a[(i + 3) * st];
        r = (((r + x0) + x1) + x2) + x3;
    }
    for (; i < n; i++) r += a[i * st];
    return r;
}
__device__ inline float pw_leaf(const float *a, int n, int st) {
    if (n < 8) return seq_sum_lds(0.f, a, n, st);
    float r0 = a[0], r1 = a[st], r2 = a[2 * st], r3 = a[3 * st];
    float r4 = a[4 * st], r5 = a[5 * st], r6 = a[6 * st], r7 = a[7 * st];
    int i = 8;
    for (; i < n - (n % 8); i += 8) {
        const float *p = a + i * st;
        r0 += p[0]; r1 += p[st]; r2 += p[2 * st]; r3 += p[3 * st];
        r4 += p[4 * st]; r5 += p[5 * st]; r6 += p[6 * st]; r7 += p[7 * st];
    }
    const float res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    return seq_sum_lds(res, a + i * st, n - i, st);
}
// both of one reduction lane's sums in one path: the sequential 0 + a[0] + a[sa] + ... (seq_sum_lds's order) and numpy's
// pairwise sum of p (n <= 128, pw_leaf's order), interleaved so that neither waits on the other's LDS round trips or
// add chain (the wave kernel's reduction lanes took the two as divergent paths, one after the other)
__device__ inline void dual_sum_lds(const float *a, int sa, const float *p, int sp, int n, float &rs, float &rp) {
    float s = 0.f;
    int i = 0;
    if (n < 8) {                                           // pairwise == sequential below 8 terms
        float q = 0.f;
        for (; i + 4 <= n; i += 4) {
            const float x0 = a[i * sa], x1 = a[(i + 1) * sa], x2 = a[(i + 2) * sa], x3 = a[(i + 3) * sa];
            const float y0 = p[i * sp], y1 = p[(i + 1) * sp], y2 = p[(i + 2) * sp], y3 = p[(i + 3) * sp];
            s = (((s + x0) + x1) + x2) + x3;
            q = (((q + y0) + y1) + y2) + y3;
        }
        for (; i < n; i++) { s += a[i * sa]; q += p[i * sp]; }
        rs = s; rp = q;
        return;
    }
    float r0 = p[0], r1 = p[sp], r2 = p[2 * sp], r3 = p[3 * sp];
    float r4 = p[4 * sp], r5 = p[5 * sp], r6 = p[6 * sp], r7 = p[7 * sp];
    for (; i < 8; i += 4) {
        const float x0 = a[i * sa], x1 = a[(i + 1) * sa], x2 = a[(i + 2) * sa], x3 = a[(i + 3) * sa];
        s = (((s + x0) + x1) + x2) + x3;
    }
    for (; i < n - (n % 8); i += 8) {
        const float *q = p + i * sp, *b = a + i * sa;
        const float x0 = b[0], x1 = b[sa], x2 = b[2 * sa], x3 = b[3 * sa];
        const float x4 = b[4 * sa], x5 = b[5 * sa], x6 = b[6 * sa], x7 = b[7 * sa];
        r0 += q[0]; r1 += q[sp]; r2 += q[2 * sp]; r3 += q[3 * sp];
        r4 += q[4 * sp]; r5 += q[5 * sp]; r6 += q[6 * sp]; r7 += q[7 * sp];
        s = (((((((s + x0) + x1) + x2) + x3) + x4) + x5) + x6) + x7;
    }
    float res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
    for (; i < n; i++) { s += a[i * sa]; res += p[i * sp]; }
    rs = s; rp = res;
}
template <int D>
__device__ inline float pw_tree(const float *a, int n, int st) {
    if (D == 0 || n <= 128) return pw_leaf(a, n, st);
    int n2 = n / 2;
    n2 -= n2 % 8;
    return pw_tree<(D > 0 ? D - 1 : 0)>(a, n2, st) + pw_tree<(D > 0 ? D - 1 : 0)>(a + n2 * st, n - n2, st);
}
// PWD = recursion levels unrolled: 0 covers n <= 128 (the common kernel), 3 covers n <= 1024.
template <int PWD>
__device__ inline float np_pairwise(const float *a, int n, int st) { return pw_tree<PWD>(a, n, st); }

__device__ inline int locate(const int *off, int n, int x) {  // largest w with off[w] <= x, w < n
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= x) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// exact idx / d for 0 <= idx < 2^24 via a float reciprocal and one correction
__device__ inline int fdiv(int idx, int d, float inv) {
    // floor(idx / d) for 0 <= idx < 2^22, inv = RN32(1/d): (idx + 1/2)/d sits at least 1/(2d) from an
    // integer, and the two float roundings move it by less than (idx + 1/2)/d * 2^-23 < 1/(2d).
    (void)d;
    return (int)(((float)idx + 0.5f) * inv);
}

// ---- exact IEEE quotients from one precomputed reciprocal (validated exhaustively-random on the host,
// scripts/check_division.c):
//  * float x / float m  ==  (float)((double)x * RN64(1/m))   for every normal quotient: the double
//    product is within 2^-52 relative of x/m, and a quotient of two 24-bit floats cannot lie that close
//    to a float rounding midpoint without being on it (it cannot be on it: it would need 25 bits);
//  * double a / double b == fma(fma(-q, b, a), y, q) with y = RN64(1/b), q = RN64(a*y)  (Markstein's
//    final correction step: y within 1/2 ulp of 1/b and q within 1 ulp of a/b -> correctly rounded).
// Non-finite operands take the plain expression (the correction would turn inf into NaN).
__device__ inline float fdiv_exact(float x, double y) { return (float)((double)x * y); }
// The operand range of the float32 quotients (Markstein's step below, and the double products fdiv_exact /
// fdiv_rcp): exact when the dividend is 0 or at least 2^-80 in magnitude and the divisor lies in [2^-20, 2^21), the
// result being finite (scripts/check_division.c case 6, 300 M random operands).  Below that the Markstein residual
// or the quotient itself leaves the normal range (x / m misrounds for some |x| < 2^-105), and a
// double product rounded to a subnormal float can sit on a rounding midpoint.  fexp is frexp's exponent (0 for 0,
// inf and NaN: zero dividends pass), so one min over fexp's tests a whole set of dividends.
constexpr int TINY_EXP = -79;   // fexp(x) >= TINY_EXP  <=>  x == 0 or |x| >= 2^-80
__device__ __forceinline__ int fexp(float x) { return __builtin_amdgcn_frexp_expf(x); }
__device__ __forceinline__ int fexp3(float a, float b, float c) { return min(min(fexp(a), fexp(b)), fexp(c)); }
__device__ __forceinline__ bool divisor_ok(float m) {   // m in [2^-20, 2^21) in magnitude
    const int e = fexp(m);
    return e >= -19 && e <= 21 && m != 0.f;
}
//  * float x / float m == fmaf(fmaf(-q, m, x), yf, q) with yf = RN32(1/m) = (float)RN64(1/m),
//    q = RN32(x*yf): the same Markstein step in binary32 (3 f32 ops, no f64 issue slots), for operands in the range
//    above; outside it (and for a zero, infinite or NaN divisor or quotient) the IEEE division.
__device__ inline float fdiv_mk(float x, float m, float yf) {
    const float q = x * yf;
    if (!__builtin_isfinite(q) || yf == 0.f) return q;
    if (__builtin_expect(fexp(x) < TINY_EXP || !divisor_ok(m), 0)) return x / m;
    return __builtin_fmaf(__builtin_fmaf(-q, m, x), yf, q);
}
__device__ inline float fxsign(float v, uint32_t s) { return __uint_as_float(__float_as_uint(v) ^ s); }
__device__ inline double dxsign(double v, uint32_t s) {
    return __hiloint2double(__double2hiint(v) ^ (int)s, __double2loint(v));
}
// Unguarded forms (finite operands and quotient): callers detect a non-finite result afterwards.
__device__ inline double ddiv_fast(double a, double b, double y) {
    const double q = a * y;
    return __builtin_fma(__builtin_fma(-q, b, a), y, q);
}
__device__ inline float fdiv_fast(float x, float m, float yf) {
    const float q = x * yf;
    return __builtin_fmaf(__builtin_fmaf(-q, m, x), yf, q);
}
__device__ inline double ddiv_exact(double a, double b, double y) {
    const double q = a * y;
    if (!__builtin_isfinite(q) || y == 0.0) return q;
    return __builtin_fma(__builtin_fma(-q, b, a), y, q);
}
// a / b for a float64 a and a b whose value is a float32 (y = RN64(1/b)): Markstein's quotient when it lands in
// [2^-800, 2^800] (scripts/check_division.c case 2; with |b| in float32 range, a and every intermediate are then
// normal doubles), a zero numerator as a * y (the IEEE sign), anything else by IEEE division.
__device__ inline double ddiv_f32d(double a, double b, double y) {
    const double q = a * y;
    const double m = __builtin_fma(__builtin_fma(-q, b, a), y, q);
    const double am = __builtin_fabs(m);
    if (__builtin_expect(am >= 0x1p-800 && am <= 0x1p800, 1)) return m;
    return a == 0.0 ? q : a / b;
}

// 1/d for a double d = (double)cur, cur a normal float: v_rcp_f64 and two Newton steps, within about
// one ulp of 1/d (not necessarily RN64(1/d)).  That suffices for the Markstein correction in
// ddiv_fast / fdiv_fast to return the correctly rounded quotient of the spring: a quotient X/cur of two
// 24-bit floats lies at least 2^-78 (relative) from every double rounding midpoint and 2^-49 from every
// float one, while the corrected value is within ~2^-100 of X/cur (tests/test_exact_division.py runs
// the same construction on the host).
__device__ __forceinline__ double rcp64_nr(double d) {
    double y = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, y, 1.0);
    y = __builtin_fma(y, e, y);
    e = __builtin_fma(-d, y, 1.0);
    return __builtin_fma(y, e, y);
}

// RN64(1/m) of a mass: for m in the divisor range (divisor_ok: the only masses whose fast quotients are used) v_rcp_f64
// and two Newton steps give the correctly rounded reciprocal — Markstein's correction from a y within one ulp is exact
// unless m's 53-bit significand is all ones, which a float32 cannot have; checked on the GPU for every float32 in
// the range, both signs (scripts/check_rcp64.hip, profiles/r04_rcp64_exhaustive.json) — 5 VALU instead of the ~12 of
// the IEEE division, and a shorter dependent chain; any other m (0, subnormal, inf, NaN, outside the range) takes the
// IEEE division, so the guarded paths see exactly what they saw before.
__device__ __forceinline__ double rcp64_nr(double d);
__device__ __forceinline__ bool divisor_ok(float m);
__device__ __forceinline__ double recip_m(float mf) {
    const double md = (double)mf;
    double y = rcp64_nr(md);
    if (__builtin_expect(!divisor_ok(mf), 0)) y = 1.0 / md;
    return y;
}

// numpy's float32 x / M for a walker's mass count M (np.mean's final division; 1 <= M < 2^20):
// (float)(x * y) with y = rcp64_nr(M) (within about an ulp of 1/M).  When x / M is a normal float, it is either
// representable or at least 2^-25 / M (relative) from every float rounding midpoint (a midpoint has a 25-bit odd
// significand), while the double product is within 2^-50 of x / M: the conversion rounds it exactly as the IEEE
// division would.  |x| < 2^-100 (a possibly subnormal quotient, where that spacing argument fails) takes the
// IEEE division, in a branch.  3 VALU instead of the ~11 of a correctly rounded float32 division.  Checked on the
// host for M < 2^11 with reciprocals up to two ulps off (scripts/check_division.c, tests/test_exact_division.py).
__device__ __forceinline__ float fdiv_count(float x, float fM, double yM) {
    float q = (float)((double)x * yM);
    if (__builtin_expect(__builtin_fabsf(x) < 0x1p-100f, 0)) q = x / fM;
    return q;
}


// numpy's float32 `x ** 2` (a scalar power: libm powf, not x*x; powf2.h): RN(x*x) unless x*x lies within 2^-32 of a
// float rounding boundary (0.29 % of floats), then glibc's algorithm restated (cold, only the lanes that need it)
__device__ __attribute__((noinline)) float np_sq_cold(float x) { return pw_pow2(x); }
// INL: the restated powf inline instead of a call — the latency-bound small-tile instances (lean NE = 1: a launch lasts
// as long as its slowest wave, and ~10 % of waves take this path): Balance-4096 -1.6 %, while the large tiles keep the
// call (canonical +1.0 % inline; profiles/r03zq_ab_sqinl_*.txt)
template <bool INL = false>
__device__ __forceinline__ float np_sq(float x) {
    float f;
    if (__builtin_expect(!pw_pow2_fast(x, &f), 0)) f = INL ? pw_pow2(x) : np_sq_cold(x);
    return f;
}
// The workgroup kernel's copy of glibc's powf tables in LDS (filled by its first 32 threads before its first barrier):
// the cold path's two dependent table reads become LDS reads instead of global loads.  In the pair passes of the
// performance_demo loop (gravity_vec's distance ** 2 for every partner) ~17 % of a wave's partner iterations take the
// cold path: with the global tables it cost 21 % of the launch (188.5 against 149.6 us with RN(x*x) everywhere,
// profiles/r04y_ab_perfdemo_sq.json).  pw_pow2's arithmetic, unchanged (powf2.h); checked on the GPU against pw_pow2
// for every float32 bit pattern (scripts/check_pow2_lanes.hip).
__shared__ double s_pw_log2[32];
__shared__ unsigned long long s_pw_exp2[32];
__device__ __forceinline__ void pw_tables_to_lds(int tid) {
    if (tid < 32) { s_pw_log2[tid] = PW_LOG2_TAB[tid]; s_pw_exp2[tid] = PW_EXP2_TAB[tid]; }
}
// (evaluated inline in the pair loop: a call ran 186.9 against 183.5 us perfdemo)
__device__ __forceinline__ float pw_pow2_lds(float x) {
    unsigned int ix = pw_asu32(x) & 0x7fffffffu;
    if (ix == 0u || ix >= 0x7f800000u) return x * x;
    if (ix < 0x00800000u) {
        ix = pw_asu32(pw_asfloat(ix) * 0x1p23f) & 0x7fffffffu;
        ix -= 23u << 23;
    }
    const unsigned int tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) & 15u);
    const unsigned int top = tmp & 0xff800000u;
    const int k = (int)top >> 23;
    const double invc = s_pw_log2[2 * i], logc = s_pw_log2[2 * i + 1];
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
    if (((pw_asu64(xd) >> 47) & 0xffffu) >= (pw_asu64(126.0) >> 47)) {
        if (xd > 0x1.fffffffd1d571p+6) return pw_asfloat(0x7f800000u);
        if (xd <= -150.0) return 0.0f;
    }
    const double shift = 0x1.8p+47;
    double kd = xd + shift;
    const unsigned long long ki = pw_asu64(kd);
    kd -= shift;
    const double rr = xd - kd;
    const unsigned long long t = s_pw_exp2[ki & 31u] + (ki << 47);
    const double sc = pw_asdouble(t);
    const double zz = PW_FMA(0x1.c6af84b912394p-5, rr, 0x1.ebfce50fac4f3p-3);
    const double rr2 = rr * rr;
    double yy = PW_FMA(0x1.62e42ff0c52d6p-1, rr, 1.0);
    yy = PW_FMA(zz, rr2, yy);
    return (float)(yy * sc);
}
// np_sq with the cold path on the LDS tables (workgroup kernel only: the tables must have been filled)
template <bool LDS_TAB>
__device__ __forceinline__ float np_sq_t(float x) {
    if (!LDS_TAB) return np_sq(x);
    float f;
    if (__builtin_expect(!pw_pow2_fast(x, &f), 0)) f = pw_pow2_lds(x);
    return f;
}

// Global -> LDS copy of n 4-byte words (16-B vector loads when both ends allow it).
template <typename T4, typename T1>
__device__ inline void stage_in(T1 *dst, const T1 *__restrict__ src, int n, int tid, int T) {
    if ((((uintptr_t)src) & 15) == 0 && (n & 3) == 0) {
        const T4 *s4 = reinterpret_cast<const T4 *>(src);
        T4 *d4 = reinterpret_cast<T4 *>(dst);
        for (int i = tid; i < (n >> 2); i += T) d4[i] = s4[i];
    } else {
        for (int i = tid; i < n; i += T) dst[i] = src[i];
    }
}
__device__ inline void stage_out(float *__restrict__ dst, const float *src, int n, int tid, int T) {
    if ((((uintptr_t)dst) & 15) == 0 && (n & 3) == 0) {
        const float4 *s4 = reinterpret_cast<const float4 *>(src);
        float4 *d4 = reinterpret_cast<float4 *>(dst);
        for (int i = tid; i < (n >> 2); i += T) d4[i] = s4[i];
    } else {
        for (int i = tid; i < n; i += T) dst[i] = src[i];
    }
}

// one 16-B spring record (wg_edge): ij = i | j << 16 | string << 31
struct EdgeRec { uint32_t ij; float rest, k, c; };
__device__ inline EdgeRec load_edge(const wg_edge *__restrict__ e, size_t i) {
    const uint4 v = reinterpret_cast<const uint4 *>(e)[i];
    return EdgeRec{v.x, __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
}
__device__ inline int edge_i(uint32_t ij) { return (int)(ij & 0x7fffu); }
__device__ inline int edge_j(uint32_t ij) { return (int)((ij >> 16) & 0x7fffu); }
__device__ inline bool edge_string(uint32_t ij) { return (ij >> 31) != 0u; }

// ------------------------------------------------------------------ per-edge and per-mass physics
// Spring term and damping force of edge `le` (block-local; masses at LDS index lm + i/j):
//   spring  gym/engine.py:78-102 resilience (two anti_forced calls, float64 force path, :73-75)
//   damping gym/optimized_walker.py:92-106 (float32), the same expression for every element type
// spring_mode 1 = the G2 element as written (gym/optimized_walker.py:48-60: float32, inverted sign).
// gt: the damping force has a component below the exact range of the mass loop's float32 quotient (fexp < TINY_EXP)
__device__ __forceinline__ void spring_edge(const EdgeRec &e, int le, int lm, float x, const float *spos,
                                            const float *svel, double *st, float *sdf, int spring_mode, bool &gt) {
    const int i = lm + edge_i(e.ij), j = lm + edge_j(e.ij);
    const float pix = spos[3 * i], piy = spos[3 * i + 1], piz = spos[3 * i + 2];
    const float pjx = spos[3 * j], pjy = spos[3 * j + 1], pjz = spos[3 * j + 2];
    const float vix = svel[3 * i], viy = svel[3 * i + 1], viz = svel[3 * i + 2];
    const float vjx = svel[3 * j], vjy = svel[3 * j + 1], vjz = svel[3 * j + 2];
    const float cur = np_norm3(pix - pjx, piy - pjy, piz - pjz);   // engine.py:86
    const float dx = cur - x;                                       // engine.py:96
    const float r0 = pjx - pix, r1 = pjy - piy, r2 = pjz - piz;     // other.pos - self.pos
    if (spring_mode == 2) {
        // G3 core.py resilience (:93-122) -> anti_forced (:85-91): the distance is float32 (:88), so the
        // force -f_size * direction / distance stays float32; no damping term.  Cold mode: IEEE divisions.
        const float fsz = (dx < 0.f && edge_string(e.ij)) ? 0.f : (-dx) * e.k;
        const float nf = -fsz;
        const float df = (CONFIG_R > (double)cur) ? (float)CONFIG_R : cur;
        st[3 * le] = (double)((nf * r0) / df); st[3 * le + 1] = (double)((nf * r1) / df);
        st[3 * le + 2] = (double)((nf * r2) / df);
        sdf[3 * le] = 0.f; sdf[3 * le + 1] = 0.f; sdf[3 * le + 2] = 0.f;
        return;
    }
    double dist = (double)cur;                                      // engine.py:73
    if (CONFIG_R > dist) dist = CONFIG_R;                           // max(distance, r)
    const double yc = 1.0 / dist;
    const float fsz = (spring_mode == 1 || !(dx < 0.f && edge_string(e.ij))) ? (-dx) * e.k : 0.f;  // :97-100
    const float nf = -fsz;                                                                           // :75
    // Fast path: Markstein quotients from one reciprocal, unguarded; exact whenever the distance is
    // unclamped and every quotient is finite (otherwise the cold branch redoes this edge with IEEE
    // divisions).  d = r / cur in float32 (optimized_walker.py:93), t = (nf * r) / dist in float64.
    const float ycf = (float)yc;
    float d0 = fdiv_fast(r0, cur, ycf), d1 = fdiv_fast(r1, cur, ycf), d2 = fdiv_fast(r2, cur, ycf);
    double t0, t1, t2;
    if (spring_mode == 1) {                                          // G2 element: float32, inverted sign
        t0 = (double)(fsz * d0); t1 = (double)(fsz * d1); t2 = (double)(fsz * d2);
    } else {
        t0 = ddiv_fast((double)(nf * r0), dist, yc);
        t1 = ddiv_fast((double)(nf * r1), dist, yc);
        t2 = ddiv_fast((double)(nf * r2), dist, yc);
    }
    // (the quotients d = r / cur are exact for r in the operand range and cur in [2^-20, 2^20))
    const bool fast_ok = cur >= 0x1p-20f && cur < 0x1p20f && fexp3(r0, r1, r2) >= TINY_EXP &&
                         (double)cur == dist && __builtin_isfinite(d0) && __builtin_isfinite(d1) &&
                         __builtin_isfinite(d2) && __builtin_isfinite(t0) && __builtin_isfinite(t1) &&
                         __builtin_isfinite(t2);
    if (__builtin_expect(!fast_ok, 0)) {
        d0 = r0; d1 = r1; d2 = r2;
        if (cur > 0.f) { d0 = r0 / cur; d1 = r1 / cur; d2 = r2 / cur; }
        if (spring_mode == 1) {
            t0 = (double)(fsz * d0); t1 = (double)(fsz * d1); t2 = (double)(fsz * d2);
        } else {
            t0 = (double)(nf * r0) / dist; t1 = (double)(nf * r1) / dist; t2 = (double)(nf * r2) / dist;
        }
    }
    st[3 * le] = t0; st[3 * le + 1] = t1; st[3 * le + 2] = t2;
    const float dk = np_dot3(vix - vjx, viy - vjy, viz - vjz, d0, d1, d2);  // :102-103
    const float dkc = dk * e.c;                                               // :104
    sdf[3 * le] = dkc * d0; sdf[3 * le + 1] = dkc * d1; sdf[3 * le + 2] = dkc * d2;
    gt = gt || fexp3(sdf[3 * le], sdf[3 * le + 1], sdf[3 * le + 2]) < TINY_EXP;
}

// One incidence entry's spring term (float64) and damping force (float32), read from LDS.
struct IncTerm { double t0, t1, t2; float f0, f1, f2; };
// Spring-term storage of a tile in LDS, every kernel: t[3 le + c] (float64), df[3 le + c] (float32).
struct TermsAoS {
    double *t;
    float *f;
    __device__ __forceinline__ IncTerm get(int le) const {
        return IncTerm{t[3 * le], t[3 * le + 1], t[3 * le + 2], f[3 * le], f[3 * le + 1], f[3 * le + 2]};
    }
    __device__ __forceinline__ void put(int le, double t0, double t1, double t2, float f0, float f1, float f2) const {
        t[3 * le] = t0; t[3 * le + 1] = t1; t[3 * le + 2] = t2;
        f[3 * le] = f0; f[3 * le + 1] = f1; f[3 * le + 2] = f2;
    }
};
template <class TS>
__device__ __forceinline__ IncTerm inc_term(const TS &ts, int lb, int ent) { return ts.get(lb + (ent >> 1)); }
// a = f32(f64(a) + t/m) (Point.forced with a float64 force, engine.py:67,75), then the damping pair
// p1.forced(-df), p2.forced(df) (optimized_walker.py:105-106); end j sees the opposite signs.
template <bool FMA_SIGN>
__device__ __forceinline__ void acc_f64_entry(const IncTerm &q, int ent, double md, double ym, float mf, float ymf,
                                              float &ax, float &ay, float &az) {
    const uint32_t sj = (uint32_t)(ent & 1) << 31;
    if (FMA_SIGN) {
        // a + (+-d) as fma(d, +-1, a): the product is exact, so the one rounding is the addition's (signed zeros
        // included), and one sign constant per end replaces an XOR per component (5 fewer VALU per entry, 5 more
        // registers: the register-tight wave kernels keep the XOR form)
        const double sgn = __hiloint2double((int)(0x3ff00000u | sj), 0);        // +1 at end i, -1 at end j
        const float sgd = __uint_as_float(0xbf800000u ^ sj);                    // damping: -1 at end i, +1 at end j
        ax = (float)__builtin_fma(ddiv_fast(q.t0, md, ym), sgn, (double)ax);
        ay = (float)__builtin_fma(ddiv_fast(q.t1, md, ym), sgn, (double)ay);
        az = (float)__builtin_fma(ddiv_fast(q.t2, md, ym), sgn, (double)az);
        ax = __builtin_fmaf(fdiv_fast(q.f0, mf, ymf), sgd, ax);
        ay = __builtin_fmaf(fdiv_fast(q.f1, mf, ymf), sgd, ay);
        az = __builtin_fmaf(fdiv_fast(q.f2, mf, ymf), sgd, az);
    } else {
        ax = (float)((double)ax + dxsign(ddiv_fast(q.t0, md, ym), sj));
        ay = (float)((double)ay + dxsign(ddiv_fast(q.t1, md, ym), sj));
        az = (float)((double)az + dxsign(ddiv_fast(q.t2, md, ym), sj));
        const uint32_t sd = sj ^ 0x80000000u;
        ax = ax + fxsign(fdiv_fast(q.f0, mf, ymf), sd);
        ay = ay + fxsign(fdiv_fast(q.f1, mf, ymf), sd);
        az = az + fxsign(fdiv_fast(q.f2, mf, ymf), sd);
    }
}

// Env forces on one mass after its spring terms, each one Point.forced in the reference's order: gravity
// [0,-g,0]/m, damp -dampk*v/m (gym/env.py:32-33, optimized_env.py:148-151), the ground penalty when below
// ground (:154-172); then Point.run1 / run2 (gym/engine.py:168-190).  a (in: spring terms) becomes old_a.
// The env forces of one mass in the reference's order, each one Point.forced: a += f/m.  FAST: the unguarded
// Markstein quotients, exact whenever every quotient is finite — a non-finite one makes the sum non-finite, and
// the caller then redoes the forces with the guarded ones (fdiv_mk, which equal IEEE division).
template <bool FAST>
__device__ __forceinline__ float fdiv_env(float x, float m, float y) { return FAST ? fdiv_fast(x, m, y) : fdiv_mk(x, m, y); }
// emin (FAST): the least fexp over the dividends, for the caller's exact-range test.
template <bool FAST>
__device__ __forceinline__ void env_forces(const KParams &kp, float mf, float ymf, float vx, float vy, float vz,
                                           float py, float &ax, float &ay, float &az, bool &hit, int &emin) {
    // the zero components of the env forces, divided by m: FAST takes Markstein's unguarded step (exact 0/m for m in
    // the divisor range, which the caller's test requires of the fast result; NaN for a tiny m, which it catches too)
    const float zm = FAST ? fdiv_fast(0.f, mf, ymf) : fdiv_mk(0.f, mf, ymf);
    // gravity [0,-g,0]/m, damp -dampk*v/m  (gym/env.py:32-33, optimized_env.py:148-151)
    const float dvx = kp.neg_dampk * vx, dvy = kp.neg_dampk * vy, dvz = kp.neg_dampk * vz;
    if (FAST) {
        emin = fexp(kp.neg_g);
        if (kp.neg_dampk != 0.f) emin = min(emin, fexp3(dvx, dvy, dvz));   // (a zero damping makes them zeros)
    }
    ax = ax + zm; ay = ay + fdiv_env<FAST>(kp.neg_g, mf, ymf); az = az + zm;
    // (a wave-uniform dampk == 0 branch adding the signed-zero dividends directly, without their quotients, measured
    // +40 VALU per wave and +0.5 % per launch: profiles/r04d_ab_canonical.json)
    ax = ax + fdiv_env<FAST>(dvx, mf, ymf);
    ay = ay + fdiv_env<FAST>(dvy, mf, ymf);
    az = az + fdiv_env<FAST>(dvz, mf, ymf);
    const float deep = py - kp.ground;
    hit = deep < 0.f;                                                // optimized_env.py:154
    if (hit) {
        const float gk = kp.neg_groundk * deep, gd = kp.neg_grounddamp * vy;
        ax = ax + zm; ay = ay + fdiv_env<FAST>(gk, mf, ymf); az = az + zm;
        ax = ax + zm; ay = ay + fdiv_env<FAST>(gd, mf, ymf); az = az + zm;
        const float ff = fabsf(deep) * kp.friction;                  // :168
        // G1 env (gym/env.py:41): [v_x*deep*friction, 0, v_z*deep*friction], left to right in float32
        const float fx = kp.friction_mode ? (vx * deep) * kp.friction : (-vx) * ff;
        const float fz = kp.friction_mode ? (vz * deep) * kp.friction : (-vz) * ff;
        if (FAST) emin = min(emin, min(fexp3(gk, gd, fx), fexp(fz)));
        ax = ax + fdiv_env<FAST>(fx, mf, ymf); ay = ay + zm; az = az + fdiv_env<FAST>(fz, mf, ymf);
    }
}

// The env forces' quotients of one mass that do not depend on ground contact (gravity, damping), which depend on m and
// v only: the barrier-free kernels compute them before the mass loop, so after it only their ordered additions and the
// contact terms remain (env_apply: env_forces<true>'s additions in the same order, bit-identical).  (All nine quotients
// ahead of the loop needed ten more registers across it: 32 B of scratch at the 6-wave budget.)
struct EnvTerms {
    float zm, eg, edx, edy, edz;   // 0/m, -g/m, the damping quotients
    int emin;                      // least fexp over their dividends (the caller's exact-range test)
};
__device__ __forceinline__ EnvTerms env_terms(const KParams &kp, float mf, float ymf, float vx, float vy, float vz) {
    EnvTerms e;
    e.zm = fdiv_fast(0.f, mf, ymf);
    const float dvx = kp.neg_dampk * vx, dvy = kp.neg_dampk * vy, dvz = kp.neg_dampk * vz;
    e.emin = fexp(kp.neg_g);
    if (kp.neg_dampk != 0.f) e.emin = min(e.emin, fexp3(dvx, dvy, dvz));
    e.eg = fdiv_fast(kp.neg_g, mf, ymf);
    e.edx = fdiv_fast(dvx, mf, ymf); e.edy = fdiv_fast(dvy, mf, ymf); e.edz = fdiv_fast(dvz, mf, ymf);
    return e;
}
__device__ __forceinline__ void env_apply(const EnvTerms &e, const KParams &kp, float mf, float ymf, float vx, float vy,
                                          float vz, float py, float &ax, float &ay, float &az, bool &hit, int &emin) {
    emin = e.emin;
    ax = ax + e.zm; ay = ay + e.eg; az = az + e.zm;
    ax = ax + e.edx; ay = ay + e.edy; az = az + e.edz;
    const float deep = py - kp.ground;
    hit = deep < 0.f;                                                // optimized_env.py:154
    if (hit) {
        const float gk = kp.neg_groundk * deep, gd = kp.neg_grounddamp * vy;
        ax = ax + e.zm; ay = ay + fdiv_fast(gk, mf, ymf); az = az + e.zm;
        ax = ax + e.zm; ay = ay + fdiv_fast(gd, mf, ymf); az = az + e.zm;
        const float ff = fabsf(deep) * kp.friction;                  // :168
        const float fx = kp.friction_mode ? (vx * deep) * kp.friction : (-vx) * ff;
        const float fz = kp.friction_mode ? (vz * deep) * kp.friction : (-vz) * ff;
        emin = min(emin, min(fexp3(gk, gd, fx), fexp(fz)));
        ax = ax + fdiv_fast(fx, mf, ymf); ay = ay + e.zm; az = az + fdiv_fast(fz, mf, ymf);
    }
}

__device__ __forceinline__ void mass_tail(const KParams &kp, float mf, float ymf, const float *p3, const float *v3,
                                          float &px, float &py, float &pz, float &vx, float &vy, float &vz,
                                          float &ax, float &ay, float &az, bool &hit, bool pinned,
                                          const EnvTerms *pre = nullptr) {
    vx = v3[0]; vy = v3[1]; vz = v3[2];
    px = p3[0]; py = p3[1]; pz = p3[2];
    if (WG_ABLATE & 256) {   // (ablation: no env forces)
        hit = py < kp.ground;
    } else if (pre) {
        // the contact-free quotients came from env_terms before the mass loop
        const float sx = ax, sy = ay, sz = az;
        int emin = 0;
        env_apply(*pre, kp, mf, ymf, vx, vy, vz, py, ax, ay, az, hit, emin);
        if (__builtin_expect(!__builtin_isfinite(ax + ay + az) || emin < TINY_EXP || !divisor_ok(mf), 0)) {
            ax = sx; ay = sy; az = sz;
            env_forces<false>(kp, mf, ymf, vx, vy, vz, py, ax, ay, az, hit, emin);
        }
    } else {
        const float sx = ax, sy = ay, sz = az;
        int emin = 0;
        env_forces<true>(kp, mf, ymf, vx, vy, vz, py, ax, ay, az, hit, emin);
        // cold: redo with exact quotients (a non-finite sum, a dividend or the mass outside the exact range)
        if (__builtin_expect(!__builtin_isfinite(ax + ay + az) || emin < TINY_EXP || !divisor_ok(mf), 0)) {
            ax = sx; ay = sy; az = sz;
            env_forces<false>(kp, mf, ymf, vx, vy, vz, py, ax, ay, az, hit, emin);
        }
    }
    if (pinned) { ax = 0.f; ay = 0.f; az = 0.f; }   // DingPoint.forced is a no-op: a stays zeros()
    // v += a*t in both integrators; the position update differs (a wave-uniform branch on the parameter, on
    // scalar locals: an if/else over px..vz references had made hipcc keep them in a stack array)
    const float nvx = vx + ax * kp.dt, nvy = vy + ay * kp.dt, nvz = vz + az * kp.dt;
    float dpx, dpy, dpz;
    if (__builtin_expect(kp.integrator == 2, 0)) {
        // Point.run2 (gym/engine.py:184-187): pos += v*t + 0.5*a*t**2 (numpy: (v*t) + ((0.5*a)*f32(t**2)))
        dpx = vx * kp.dt + (0.5f * ax) * kp.dt2;
        dpy = vy * kp.dt + (0.5f * ay) * kp.dt2;
        dpz = vz * kp.dt + (0.5f * az) * kp.dt2;
    } else {
        // Point.run1 (gym/engine.py:174-178): pos += v_new*t
        dpx = nvx * kp.dt; dpy = nvy * kp.dt; dpz = nvz * kp.dt;
    }
    px = px + dpx; py = py + dpy; pz = pz + dpz;
    vx = nvx; vy = nvy; vz = nvz;
}

// Mass `lp`: the ordered force accumulation over its incidence list (edge order, spring then damping
// per edge — gym/optimized_walker.py:124-127 with gym/engine.py:65-76, 101-102), then gravity, linear
// damping and the ground penalty (gym/env.py:31-41 / gym/optimized_env.py:146-172, each one
// Point.forced), then Point.run1 (gym/engine.py:174-178).  Returns the new state and old_a.
template <class TS, bool FMA_SIGN = true>
__device__ __forceinline__ void mass_accumulate(const TS &ts, const uint16_t *inc, int lb, int s0, int s1, float mf,
                                                float &ax, float &ay, float &az, int spring_mode, bool force = false) {
    const double md = (double)mf;
    const double ym = 1.0 / md;      // one IEEE division per mass; every /m below is exact from it
    const float ymf = (float)ym;     // = RN32(1/m)
    ax = 0.f; ay = 0.f; az = 0.f;
    // Both ends of an edge see the same spring term t and damping force df with opposite signs; the
    // divisions are odd functions (RN is sign-symmetric), so the quotient is formed once and its sign
    // flipped by one XOR: -(t/m) == (-t)/m exactly, a + (-d) == a - d.
    if (spring_mode == 1) {
        for (int r = s0; r < s1; r++) {
            const int ent = inc[r];
            const int le = lb + (ent >> 1);
            const uint32_t sj = (uint32_t)(ent & 1) << 31;   // sign of the spring term at this end
            const IncTerm q = ts.get(le);
            ax = ax + fxsign(fdiv_mk((float)q.t0, mf, ymf), sj);
            ay = ay + fxsign(fdiv_mk((float)q.t1, mf, ymf), sj);
            az = az + fxsign(fdiv_mk((float)q.t2, mf, ymf), sj);
            const uint32_t sd = sj ^ 0x80000000u;          // damping: p1 gets -df, p2 gets +df
            ax = ax + fxsign(fdiv_mk(q.f0, mf, ymf), sd);
            ay = ay + fxsign(fdiv_mk(q.f1, mf, ymf), sd);
            az = az + fxsign(fdiv_mk(q.f2, mf, ymf), sd);
        }
    } else {
        // Fast path: the Markstein quotients without their non-finite guards.  They differ from the
        // IEEE quotient only when q = t*RN(1/m) is not finite, and then the running sum becomes (and
        // stays) inf/NaN — so a finite result proves every quotient was exact.  A lane whose result is
        // not finite redoes its list with plain IEEE divisions (wave-uniform branch, cold).
        // Software-pipelined, two register sets (A, B) in ping-pong: the reads of the next entry are
        // issued before the arithmetic of the current one, so LDS latency overlaps it.  Reads past the
        // list end are clamped to its last entry (always a valid address) and their values unused.
        if (s1 > s0) {
            const int rl = s1 - 1;
            int ea = inc[s0], eb = inc[min(s0 + 1, rl)];
            IncTerm A = inc_term(ts, lb, ea), B;
            for (int r = s0; r < s1; r += 2) {
                B = inc_term(ts, lb, eb);
                const int ea2 = inc[min(r + 2, rl)];
                __builtin_amdgcn_sched_barrier(0);   // keep the reads above the arithmetic
                acc_f64_entry<FMA_SIGN>(A, ea, md, ym, mf, ymf, ax, ay, az);
                if (r + 1 >= s1) break;
                A = inc_term(ts, lb, ea2);
                const int eb2 = inc[min(r + 3, rl)];
                __builtin_amdgcn_sched_barrier(0);
                acc_f64_entry<FMA_SIGN>(B, eb, md, ym, mf, ymf, ax, ay, az);
                ea = ea2; eb = eb2;
                // opaque hand-over: stops the phi-of-loads fold that would sink A's reads to its use
                asm volatile("" : "+v"(A.t0), "+v"(A.t1), "+v"(A.t2), "+v"(A.f0), "+v"(A.f1), "+v"(A.f2), "+v"(ea), "+v"(eb));
            }
        }
        // force: a damping force of the tile outside the exact range of the float32 quotient (the caller's flag), or a
        // mass outside its divisor range
        const bool bad = force || !divisor_ok(mf) ||
                         !(__builtin_isfinite(ax) && __builtin_isfinite(ay) && __builtin_isfinite(az));
        if (__builtin_expect(bad, 0)) {
            ax = 0.f; ay = 0.f; az = 0.f;
            for (int r = s0; r < s1; r++) {
                const int ent = inc[r];
                const int le = lb + (ent >> 1);
                const uint32_t sj = (uint32_t)(ent & 1) << 31;
                const IncTerm q = ts.get(le);
                ax = (float)((double)ax + dxsign(q.t0 / md, sj));
                ay = (float)((double)ay + dxsign(q.t1 / md, sj));
                az = (float)((double)az + dxsign(q.t2 / md, sj));
                const uint32_t sd = sj ^ 0x80000000u;
                ax = ax + fxsign(q.f0 / mf, sd);
                ay = ay + fxsign(q.f1 / mf, sd);
                az = az + fxsign(q.f2 / mf, sd);
            }
        }
    }
}

// The barrier-free kernels' mass loop (spring_mode 0), with the per-entry bookkeeping cut to five VALU: an entry
// (edge << 1 | end) addresses its term records as tb + 24 * edge and fb + 12 * edge (two v_mad_u32_u24 from the
// walker's term bases), its end's sign is one v_lshl_or_b32 into the float64 and one into the float32 +-1 (the
// damping takes the opposite sign through the fma's neg modifier), and the list is walked by pointer with no
// clamp on the read-ahead: the entries after a mass's list are the next mass's, and the tile's last list is
// followed by a zero word (the wave writes one after its incidence words), so every read-ahead is a valid entry
// whose values go unused.  Arithmetic and its order are those of acc_f64_entry<true> (bit-identical).
__device__ __forceinline__ IncTerm inc_term_at(const char *tb, const char *fb, uint32_t ent) {
    const uint32_t e = ent >> 1;
    const double *t = reinterpret_cast<const double *>(tb + __umul24(e, 24u));
    const float *f = reinterpret_cast<const float *>(fb + __umul24(e, 12u));
    return IncTerm{t[0], t[1], t[2], f[0], f[1], f[2]};
}
__device__ __forceinline__ void acc_entry_v2(const IncTerm &q, uint32_t ent, double md, double ym, float mf, float ymf,
                                             float &ax, float &ay, float &az) {
    // +1 at end i, -1 at end j, as the float64's high word and as a float32 (the damping takes -sgf); one
    // v_lshl_or_b32 each (the compiler would share one shift between two ors)
    uint32_t hi, sf;
    asm("v_lshl_or_b32 %0, %1, 31, %2" : "=v"(hi) : "v"(ent), "s"(0x3ff00000u));
    asm("v_lshl_or_b32 %0, %1, 31, %2" : "=v"(sf) : "v"(ent), "s"(0x3f800000u));
    const double sgn = __hiloint2double((int)hi, 0);
    const float sgf = __uint_as_float(sf);
    ax = (float)__builtin_fma(ddiv_fast(q.t0, md, ym), sgn, (double)ax);
    ay = (float)__builtin_fma(ddiv_fast(q.t1, md, ym), sgn, (double)ay);
    az = (float)__builtin_fma(ddiv_fast(q.t2, md, ym), sgn, (double)az);
    ax = __builtin_fmaf(fdiv_fast(q.f0, mf, ymf), -sgf, ax);
    ay = __builtin_fmaf(fdiv_fast(q.f1, mf, ymf), -sgf, ay);
    az = __builtin_fmaf(fdiv_fast(q.f2, mf, ymf), -sgf, az);
}
// ym = RN64(1/m) from the caller (one IEEE division per mass, shared with the env forces)
__device__ __forceinline__ void mass_accumulate_v2(const TermsAoS &ts, const uint16_t *inc, int lb, int s0, int s1,
                                                   float mf, double ym, float &ax, float &ay, float &az, bool force) {
    const double md = (double)mf;
    const float ymf = (float)ym;      // = RN32(1/m)
    ax = 0.f; ay = 0.f; az = 0.f;
    const char *tb = reinterpret_cast<const char *>(ts.t + 3 * lb), *fb = reinterpret_cast<const char *>(ts.f + 3 * lb);
    if (s1 > s0) {
        const uint16_t *p = inc + s0;
        uint32_t ea = p[0], eb = p[1];
        IncTerm A = inc_term_at(tb, fb, ea), B;
        for (int r = s0; r < s1; r += 2) {
            B = inc_term_at(tb, fb, eb);
            const uint32_t ea2 = p[2];
            __builtin_amdgcn_sched_barrier(0);   // keep the reads above the arithmetic (without, at NE = 1: +2.5 %,
                                                 // profiles/r06h_ab_nosb_balance4096.json)
            acc_entry_v2(A, ea, md, ym, mf, ymf, ax, ay, az);
            if (r + 1 >= s1) break;
            A = inc_term_at(tb, fb, ea2);
            const uint32_t eb2 = p[3];
            __builtin_amdgcn_sched_barrier(0);
            acc_entry_v2(B, eb, md, ym, mf, ymf, ax, ay, az);
            ea = ea2; eb = eb2; p += 2;
            asm volatile("" : "+v"(A.t0), "+v"(A.t1), "+v"(A.t2), "+v"(A.f0), "+v"(A.f1), "+v"(A.f2));
        }
    }
    // a non-finite sum (some quotient was not exact, or an input not finite), a damping force of the wave outside the
    // float32 quotient's exact range (force), or a mass outside its divisor range: redo the list with IEEE divisions
    if (__builtin_expect(force || !divisor_ok(mf) ||
                         !(__builtin_isfinite(ax) && __builtin_isfinite(ay) && __builtin_isfinite(az)), 0)) {
        ax = 0.f; ay = 0.f; az = 0.f;
        for (int r = s0; r < s1; r++) {
            const int ent = inc[r];
            const uint32_t sj = (uint32_t)(ent & 1) << 31;
            const IncTerm q = ts.get(lb + (ent >> 1));
            ax = (float)((double)ax + dxsign(q.t0 / md, sj));
            ay = (float)((double)ay + dxsign(q.t1 / md, sj));
            az = (float)((double)az + dxsign(q.t2 / md, sj));
            const uint32_t sd = sj ^ 0x80000000u;
            ax = ax + fxsign(q.f0 / mf, sd);
            ay = ay + fxsign(q.f1 / mf, sd);
            az = az + fxsign(q.f2 / mf, sd);
        }
    }
}

// spring_mode 2: one mass of the G3 engine, Environment.update_physics (gym/optimized_walker/env.py:135-184),
// all float32 with IEEE divisions: a = 0 + (gravity*m)/m (:141-146), the spring terms in edge order
// (:149-150), v *= damping (:153-154), drag ((-0.5*air)*|v|)*v / m (:157-161), Point.run1 (core.py:185-200),
// then the position-clamp ground with restitution and friction (:164-178).  A DingPoint (pinned) is not one
// of the env's points: no force, no damping, no ground, but run1 still moves it by its velocity.
__device__ __forceinline__ void g3_mass_step(const KParams &kp, const double *st, const uint16_t *inc, int lb, int s0,
                                          int s1, float mf, const float *p3, const float *v3, float &px, float &py,
                                          float &pz, float &vx, float &vy, float &vz, float &ax, float &ay,
                                          float &az, bool &hit, bool pinned) {
    ax = 0.f; ay = 0.f; az = 0.f;
    vx = v3[0]; vy = v3[1]; vz = v3[2];
    if (!pinned) {
        ax = 0.f + (kp.g3g[0] * mf) / mf; ay = 0.f + (kp.g3g[1] * mf) / mf; az = 0.f + (kp.g3g[2] * mf) / mf;
        for (int r = s0; r < s1; r++) {
            const int ent = inc[r];
            const int le = lb + (ent >> 1);
            const uint32_t sj = (uint32_t)(ent & 1) << 31;   // end j: direction and term negated exactly
            ax = ax + fxsign((float)st[3 * le] / mf, sj);
            ay = ay + fxsign((float)st[3 * le + 1] / mf, sj);
            az = az + fxsign((float)st[3 * le + 2] / mf, sj);
        }
        vx = vx * kp.g3_damp; vy = vy * kp.g3_damp; vz = vz * kp.g3_damp;
        const float coef = kp.g3_dragc * np_norm3(vx, vy, vz);
        ax = ax + (coef * vx) / mf; ay = ay + (coef * vy) / mf; az = az + (coef * vz) / mf;
    }
    vx = vx + ax * kp.dt; vy = vy + ay * kp.dt; vz = vz + az * kp.dt;
    px = p3[0] + vx * kp.dt; py = p3[1] + vy * kp.dt; pz = p3[2] + vz * kp.dt;
    hit = !pinned && kp.g3_ground && py <= kp.g3_level;
    if (hit) {
        py = kp.g3_level;
        if (vy < 0.f) { vy = (-vy) * kp.g3_rest; vx = vx * kp.g3_fric; vz = vz * kp.g3_fric; }
    }
}

__device__ __forceinline__ void mass_step(const KParams &kp, const double *st, const float *sdf,
                                          const uint16_t *inc, int lb, int s0, int s1, float mf,
                                          const float *p3, const float *v3, float &px, float &py, float &pz,
                                          float &vx, float &vy, float &vz, float &ax, float &ay, float &az,
                                          bool &hit, int spring_mode, bool pinned, bool force) {
    if (spring_mode == 2) {
        g3_mass_step(kp, st, inc, lb, s0, s1, mf, p3, v3, px, py, pz, vx, vy, vz, ax, ay, az, hit, pinned);
        return;
    }
    mass_accumulate(TermsAoS{const_cast<double *>(st), const_cast<float *>(sdf)}, inc, lb, s0, s1, mf, ax, ay, az,
                    spring_mode, force);
    const float ymf = (float)(1.0 / (double)mf);
    mass_tail(kp, mf, ymf, p3, v3, px, py, pz, vx, vy, vz, ax, ay, az, hit, pinned);
}

// ------------------------------------------------------------------ cross-lane reductions
// A walker's M masses are M adjacent lanes of one wave when M divides 64 (uniform batches): numpy's
// summation orders are then reproduced in registers with ds_bpermute shuffles — no LDS round trip,
// no extra barrier (north_star: "wavefront shuffles for per-walker reductions").
__device__ inline float lane_get(float v, int src) { return __shfl(v, src, 64); }

// DPP lane moves (one VALU source modifier, no LDS traffic): row_shr:1 0x111, row_ror:8 0x128,
// wave_shr:1 0x138, quad_perm [1,0,3,2] 0xB1 / [2,3,0,1] 0x4E, row_half_mirror 0x141.
template <int CTRL> __device__ inline float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}

// Sequential float sums ((0 + x_0) + x_1) + ... + x_{M-1} over the walker's M lanes, three at once.
// Chain: s_q <- s_{q-1} + x_q repeated M-1 times leaves lane base+M-1 holding exactly that left-to-right
// sum of its own walker (the chain never leaves the walker's lanes); then one broadcast per sum.
// One chain per loop: three chains in one loop body get SLP-packed into v_pk_add_f32, which cannot take a DPP
// operand (2 moves + 2 zero fills + 1 packed add for two chains instead of 2 v_add_f32_dpp).
template <int CTRL>
__device__ inline float seq_chain(float x, int M) {
    float a = 0.f + x;
    for (int t = 1; t < M; t++) a = dpp_f<CTRL>(a) + x;
    return a;
}
// M == 4 (Balance-v0, Box-v0): a walker is one DPP quad, so every lane of it adds the quad's four values in order
// from quad_perm broadcasts: ((0 + x_0) + x_1) + x_2) + x_3 in every lane, no LDS round trip (the step of a small
// batch is one wave's latency chain).
template <int K> __device__ inline float quad_bcast(float v) { return dpp_f<K | (K << 2) | (K << 4) | (K << 6)>(v); }
__device__ inline float seq_sum_quad(float x) {
    float a = 0.f + quad_bcast<0>(x);
    a = a + quad_bcast<1>(x);
    a = a + quad_bcast<2>(x);
    return a + quad_bcast<3>(x);
}
__device__ inline void seq_sum3_lanes(float x, float y, float z, int base, int M, float &sx, float &sy, float &sz) {
    float a, b, c;
    if (M == 4) {
        sx = seq_sum_quad(x); sy = seq_sum_quad(y); sz = seq_sum_quad(z);
        return;
    }
    if (M == 16) {
        // the three chains interleaved in one unrolled body (three independent DPP adds per step instead of one chain
        // at a time behind a scalar loop); the empty asm keeps each chain's adds scalar (no SLP packing, which has
        // no DPP form)
        a = 0.f + x; b = 0.f + y; c = 0.f + z;
#pragma unroll
        for (int t = 1; t < 16; t++) {
            a = dpp_f<0x111>(a) + x; b = dpp_f<0x111>(b) + y; c = dpp_f<0x111>(c) + z;
            asm volatile("" : "+v"(a), "+v"(b), "+v"(c));
        }
    } else if (M <= 16) {     // walkers of M | 16 lanes sit inside one 16-lane DPP row
        a = seq_chain<0x111>(x, M); b = seq_chain<0x111>(y, M); c = seq_chain<0x111>(z, M);
    } else {
        a = seq_chain<0x138>(x, M); b = seq_chain<0x138>(y, M); c = seq_chain<0x138>(z, M);
    }
    const int last = base + M - 1;
    sx = lane_get(a, last); sy = lane_get(b, last); sz = lane_get(c, last);
}
__device__ inline float seq_sum_lanes(float x, int base, int M) {
    if (M == 4) return seq_sum_quad(x);
    float a, b, c;
    seq_sum3_lanes(x, 0.f, 0.f, base, M, a, b, c);
    return a;
}
// numpy pairwise sum over the walker's M lanes (M divides 64): < 8 sequential; otherwise 8 interleaved
// partial sums r_j = x_j + x_{j+8} + ... then ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)).  For M = 8, 16 the
// partials and the tree are DPP moves (row_ror:8, then quad_perm xor-1, xor-2 and row_half_mirror,
// which pairs each lane of one 4-lane half with a lane of the other: IEEE addition is commutative).
__device__ inline float pw_sum_lanes(float x, int base, int M, int lane) {
    if (M < 8) return seq_sum_lanes(x, base, M);
    if (M <= 16) {
        float r = (M == 16) ? x + dpp_f<0x128>(x) : x;
        r = r + dpp_f<0xB1>(r);
        r = r + dpp_f<0x4E>(r);
        return r + dpp_f<0x141>(r);
    }
    const int j = (lane - base) & 7;
    float r = lane_get(x, base + j);
    for (int k = 8; k < M; k += 8) r += lane_get(x, base + j + k);
    r = r + __shfl_xor(r, 1, 64);
    r = r + __shfl_xor(r, 2, 64);
    r = r + __shfl_xor(r, 4, 64);
    return r;
}

// All seven per-walker sums of the observe step (lane values -> per-walker totals): the sequential sums of x, y, z
// (getstat's mid, info's centroid) and numpy's pairwise sums of y (np.mean), |v|, m|v|^2, m g (y - ground).  For
// M = 4 and M = 16 (Balance-v0 / Box-v0 and the canonical walker) the seven chains run interleaved in one
// straight-line block — every DPP add has six independent ones to fill its wait states, where the generic path
// (M known only at run time) runs each sum behind its own branches — with the same additions in the same order.
struct WalkerSums { float sx, sy, sz, ysum, vsum, ksum, psum; };
#define WG_OPAQUE7(a, b, c, d, e, f, g) asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e), "+v"(f), "+v"(g))
__device__ inline WalkerSums walker_sums(float px, float py, float pz, float nv, float ke, float pe, int base, int M,
                                         int lane) {
    WalkerSums r;
    if (M == 4) {
        // a walker is one DPP quad: every lane adds the quad's four values in order (M < 8: pairwise == sequential)
        // (x_0 + 0 with the zero in a register: one v_add_f32_dpp each, no separate DPP move; x + 0 == 0 + x)
        float z = 0.f;
        asm volatile("" : "+v"(z));
        float a = quad_bcast<0>(px) + z, b = quad_bcast<0>(py) + z, c = quad_bcast<0>(pz) + z;
        float d = quad_bcast<0>(nv) + z, e = quad_bcast<0>(ke) + z, f = quad_bcast<0>(pe) + z;
        WG_OPAQUE7(a, b, c, d, e, f, py);
        a = a + quad_bcast<1>(px); b = b + quad_bcast<1>(py); c = c + quad_bcast<1>(pz);
        d = d + quad_bcast<1>(nv); e = e + quad_bcast<1>(ke); f = f + quad_bcast<1>(pe);
        WG_OPAQUE7(a, b, c, d, e, f, py);
        a = a + quad_bcast<2>(px); b = b + quad_bcast<2>(py); c = c + quad_bcast<2>(pz);
        d = d + quad_bcast<2>(nv); e = e + quad_bcast<2>(ke); f = f + quad_bcast<2>(pe);
        WG_OPAQUE7(a, b, c, d, e, f, py);
        // (one add at a time behind an empty asm: otherwise SLP pairs the last step's adds into v_pk_add_f32, which takes
        // no DPP operand, and each pair costs two DPP moves more)
        a = a + quad_bcast<3>(px); asm volatile("" : "+v"(a));
        b = b + quad_bcast<3>(py); asm volatile("" : "+v"(b));
        c = c + quad_bcast<3>(pz); asm volatile("" : "+v"(c));
        d = d + quad_bcast<3>(nv); asm volatile("" : "+v"(d));
        e = e + quad_bcast<3>(ke); asm volatile("" : "+v"(e));
        f = f + quad_bcast<3>(pe);
        r.sx = a; r.sy = b; r.sz = c; r.ysum = b; r.vsum = d; r.ksum = e; r.psum = f;
        return r;
    }
    if (M == 16) {
        // sequential: s_q <- s_{q-1} + x_q along the row (lane base + 15 ends with the walker's left-to-right sum);
        // pairwise: r_j = x_j + x_{j+8}, then ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) by quad_perm / half-mirror moves
        float a = 0.f + px, b = 0.f + py, c = 0.f + pz;
        float y = py + dpp_f<0x128>(py), v = nv + dpp_f<0x128>(nv), k = ke + dpp_f<0x128>(ke), e = pe + dpp_f<0x128>(pe);
        WG_OPAQUE7(a, b, c, y, v, k, e);
        y = y + dpp_f<0xB1>(y); v = v + dpp_f<0xB1>(v); k = k + dpp_f<0xB1>(k); e = e + dpp_f<0xB1>(e);
        WG_OPAQUE7(a, b, c, y, v, k, e);
        y = y + dpp_f<0x4E>(y); v = v + dpp_f<0x4E>(v); k = k + dpp_f<0x4E>(k); e = e + dpp_f<0x4E>(e);
        WG_OPAQUE7(a, b, c, y, v, k, e);
        // (the last step one add at a time: SLP would pair them into v_pk_add_f32, two DPP moves per pair)
        y = y + dpp_f<0x141>(y); asm volatile("" : "+v"(y));
        v = v + dpp_f<0x141>(v); asm volatile("" : "+v"(v));
        k = k + dpp_f<0x141>(k); asm volatile("" : "+v"(k));
        e = e + dpp_f<0x141>(e); asm volatile("" : "+v"(e));
#pragma unroll
        for (int t = 1; t < 16; t++) {
            a = dpp_f<0x111>(a) + px; b = dpp_f<0x111>(b) + py; c = dpp_f<0x111>(c) + pz;
            asm volatile("" : "+v"(a), "+v"(b), "+v"(c));
        }
        const int last = base + 15;
        r.sx = lane_get(a, last); r.sy = lane_get(b, last); r.sz = lane_get(c, last);
        r.ysum = y; r.vsum = v; r.ksum = k; r.psum = e;
        return r;
    }
    seq_sum3_lanes(px, py, pz, base, M, r.sx, r.sy, r.sz);
    r.ysum = pw_sum_lanes(py, base, M, lane); r.vsum = pw_sum_lanes(nv, base, M, lane);
    r.ksum = pw_sum_lanes(ke, base, M, lane); r.psum = pw_sum_lanes(pe, base, M, lane);
    return r;
}
#undef WG_OPAQUE7

// ------------------------------------------------------------------ pair terms
// One gravity / coulomb partner (gym/engine.py:128-147 -> anti_forced :69-76 -> forced :65-67), all float64:
// r = max(norm(d) as float64, Config.r); f = -c*s_lo*s_hi / r**2; a = f32(f64(a) + ((-f)*d / r) / m).  The
// divisions by r (when unclamped: a float32 value) and by m go through ddiv_f32d with one IEEE reciprocal each.
__device__ __forceinline__ void pair_central_term(double coef, double slo, double shi, float d0, float d1, float d2,
                                                  double md, double ym, float &ax, float &ay, float &az) {
    const double cur = (double)np_norm3(d0, d1, d2);   // == norm(p_i - p_j): the squares do not see the sign
    const double r = CONFIG_R > cur ? CONFIG_R : cur;
    const double f = ((-coef) * slo) * shi / (r * r);
    const double nf = -f;
    double t0 = nf * (double)d0, t1 = nf * (double)d1, t2 = nf * (double)d2;
    if (__builtin_expect(r == cur, 1)) {
        const double yr = 1.0 / r;
        t0 = ddiv_f32d(t0, r, yr); t1 = ddiv_f32d(t1, r, yr); t2 = ddiv_f32d(t2, r, yr);
    } else {                                           // clamped (or NaN) distance: IEEE
        t0 = t0 / r; t1 = t1 / r; t2 = t2 / r;
    }
    ax = (float)((double)ax + ddiv_f32d(t0, md, ym));
    ay = (float)((double)ay + ddiv_f32d(t1, md, ym));
    az = (float)((double)az + ddiv_f32d(t2, md, ym));
}
// a / b by Markstein's correction from y ~ 1/b, written -(-r*y - q) so that a = +-0 gives the IEEE signed zero
__device__ __forceinline__ double mk_div(double a, double b, double y) {
    const double q = a * y;
    const double r = __builtin_fma(-q, b, a);
    return -__builtin_fma(-r, y, -q);
}
// pair_central_term without IEEE divisions or the compiler's sqrtf: the correctly rounded sqrt of a float in
// [2^-96, 2^126) (sqrt_mid); f / r^2 from rcp64_nr(r^2) and Markstein's step (the compiler's own double division
// minus the operand scaling, which no operand in the range admitted here needs); RN64(1/r) as one Newton step
// from r * y2 (r is a float32 value: 1/r lies >= 2^-77 (relative) from every double rounding midpoint, the
// step lands within ~2^-100); the divisions by r and m as ddiv_f32d's Markstein quotients.  bad is raised for
// a distance outside that range or |f| < 2^-600 (zero included: every later numerator is then >= 2^-812 in
// magnitude or exactly zero, so no residual underflows); a non-finite quotient makes the sum non-finite.  The
// caller redoes the partner loop with pair_central_term when bad is set or the sum is not finite.
__device__ __forceinline__ void pair_central_fast(double coef, double slo, double shi, float d0, float d1, float d2,
                                                  double md, double ym, float &ax, float &ay, float &az, bool &bad) {
    const float sq = (float)(((double)(d0 * d0) + (double)(d1 * d1)) + (double)(d2 * d2));   // np_norm3's sum
    const double r = (double)sqrt_mid(sq);             // >= 2^-48 > Config.r: max(distance, r) is the distance
    const double r2 = r * r;
    const double y2 = rcp64_nr(r2);
    const double f = mk_div(((-coef) * slo) * shi, r2, y2);
    const double yr0 = r * y2;
    const double yr = __builtin_fma(yr0, __builtin_fma(-r, yr0, 1.0), yr0);
    const double nf = -f;
    ax = (float)((double)ax + mk_div(mk_div(nf * (double)d0, r, yr), md, ym));
    ay = (float)((double)ay + mk_div(mk_div(nf * (double)d1, r, yr), md, ym));
    az = (float)((double)az + mk_div(mk_div(nf * (double)d2, r, yr), md, ym));
    const uint32_t fe = ((uint32_t)__double2hiint(f) >> 20) & 0x7ffu;
    bad = bad || !(sq >= 0x1p-96f && sq < 0x1p126f) || fe < 1023u - 600u;
}

// One colliding bounce partner: resilience(i, r_s + r_i, k/2) seen from this end (gym/engine.py:78-102), the
// float64 force path with the float32 numerator nf * d.
__device__ __forceinline__ void bounce_term(float cur, float nf, float d0, float d1, float d2, double md, double ym,
                                            float &ax, float &ay, float &az) {
    const double dc = (double)cur;
    const double dist = CONFIG_R > dc ? CONFIG_R : dc;
    double t0 = (double)(nf * d0), t1 = (double)(nf * d1), t2 = (double)(nf * d2);
    if (__builtin_expect(dist == dc, 1)) {
        const double yd = 1.0 / dist;
        t0 = ddiv_f32d(t0, dist, yd); t1 = ddiv_f32d(t1, dist, yd); t2 = ddiv_f32d(t2, dist, yd);
    } else {
        t0 = t0 / dist; t1 = t1 / dist; t2 = t2 / dist;
    }
    ax = (float)((double)ax + ddiv_f32d(t0, md, ym));
    ay = (float)((double)ay + ddiv_f32d(t1, md, ym));
    az = (float)((double)az + ddiv_f32d(t2, md, ym));
}

// One partner of G2 Point.gravity = Point.gravity_vec (gym/optimized_engine.py:167-193, the N-body of the performance_demo
// loop, gym/performance_demo.py:52-58), seen from mass q, all float32 as numpy evaluates it: distance =
// norm(p_j - p_i) WITHOUT .astype(float) (:185-186: a numpy float32); max(distance, Config.r); f = -Config.g * m_i * m_j
// / distance ** 2 (:189: the Python-float numerator weakly cast to float32, distance ** 2 numpy's float32 power =
// libm powf, np_sq); force = f * direction / distance (:192, float32); p_i.forced(force), p_j.forced(-force)
// (:193-194, a += force / m in float32).  d = partner - self: q receives (f * d) / distance from either role (the
// negations are exact).  cg = f32(-Config.g * m_lo * m_hi) from the Python product (numerator in float64).  A
// distance below Config.r leaves the Python float 16e-36 in its place: f and the division then go through its
// float32 casts (:189-192 with a Python-float distance).
// The reference arithmetic of one partner (IEEE float32 divisions and sqrtf): the three quotients force_c / m.
__device__ __forceinline__ void g2_gravity_cold(double cgd, float d0, float d1, float d2, float mf, float &q0, float &q1,
                                             float &q2) {
    const float dist = np_norm3(d0, d1, d2);
    float f, dv;
    if (!(CONFIG_R > (double)dist)) {        // unclamped (NaN too: max keeps the float32 NaN)
        f = (float)cgd / pw_pow2(dist);
        dv = dist;
    } else {
        f = (float)(cgd / (CONFIG_R * CONFIG_R));   // Python floats throughout, cast where they meet float32
        dv = (float)CONFIG_R;
    }
    q0 = ((f * d0) / dv) / mf;
    q1 = ((f * d1) / dv) / mf;
    q2 = ((f * d2) / dv) / mf;
}
// RN32(a / b) for a float32 a and b from y ~ 1/b (rcp64_nr, within ~1 ulp of a double): the double product a * y lies
// within 2^-51 (relative) of a / b, and a quotient of two 24-bit floats that is a normal float32 is at least 2^-47
// from every float32 rounding midpoint, so the one rounding to float32 is RN32(a / b); zero, inf and NaN numerators
// propagate as IEEE division does.  A subnormal quotient can sit ON a midpoint (x / 6 for x = odd * 3 * 2^-149): the
// callers keep the operands in the exact range (TINY_EXP), which keeps every quotient normal.
__device__ __forceinline__ float fdiv_rcp(float a, double y) { return (float)((double)a * y); }
// G2 gravity_vec partner, fast form: np_norm3's sum, sqrt_mid, numpy's distance ** 2 (np_sq: RN(x*x) or, for the
// 0.29 % of distances near a rounding boundary, the restated powf), the four quotients by fdiv_rcp from two
// reciprocals, the division by m from ym = RN64(1/m) (fdiv_exact).  ok = false when the squared distance leaves
// [2^-96, 2^126) (sqrt_mid's range, which also keeps the distance clear of Config.r); the caller then takes
// g2_gravity_cold for this partner.
template <bool LDS_TAB = false>
__device__ __forceinline__ void g2_gravity_fast(float cg, float d0, float d1, float d2, double ym, float &q0,
                                                float &q1, float &q2, bool &ok) {
    const float sq = (float)(((double)(d0 * d0) + (double)(d1 * d1)) + (double)(d2 * d2));
    const float dist = sqrt_mid(sq);
    const float dd = np_sq_t<LDS_TAB>(dist);
    const float f = fdiv_rcp(cg, rcp64_nr((double)dd));
    const double yd = rcp64_nr((double)dist);
    const float e0 = f * d0, e1 = f * d1, e2 = f * d2;
    // the exact range: distance in [2^-20, 2^20) (inside sqrt_mid's range), the dividends cg and f * d either 0 or at
    // least 2^-80: every quotient (cg / dd, e / dist, then / m with m in its divisor range) is then a normal float32
    ok = sq >= 0x1p-40f && sq < 0x1p40f && min(fexp(cg), fexp3(e0, e1, e2)) >= TINY_EXP;
    q0 = fdiv_exact(fdiv_rcp(e0, yd), ym);
    q1 = fdiv_exact(fdiv_rcp(e1, yd), ym);
    q2 = fdiv_exact(fdiv_rcp(e2, yd), ym);
}
template <bool LDS_TAB = false>
__device__ __forceinline__ void g2_gravity_term(double cgd, float d0, float d1, float d2, float mf, double ym,
                                                float &ax, float &ay, float &az) {
    float q0, q1, q2;
    bool ok;
    g2_gravity_fast<LDS_TAB>((float)cgd, d0, d1, d2, ym, q0, q1, q2, ok);
    if (__builtin_expect(!ok || !divisor_ok(mf), 0)) g2_gravity_cold(cgd, d0, d1, d2, mf, q0, q1, q2);
    ax = ax + q0;
    ay = ay + q1;
    az = az + q2;
}

// ------------------------------------------------------------------ pair passes from LDS (workgroup kernel)
// SURVEY §8(f) 3 for walkers the lean kernel does not take (M not dividing 64, M > 64, ragged batches): the
// arithmetic of pair_central / pair_bounce (lean kernel, below) with the partners' positions read from the tile's
// LDS copy, unchanged until every mass of the tile has accumulated (walker_step_kernel puts a barrier there).
// Point.electrostatic (gym/engine.py:150-158) of mass q: for every other point i in registry order, r = max(norm(p_q -
// p_i) as float64, Config.r), f = -Config.k * e_q * e_i / r**2 (self's charge first, unlike coulomb's lower index
// first), then q.anti_forced(f, i): only q receives, (-f) * (p_i - p_q) / r in float64, divided by m.  The same
// partner arithmetic as the coulomb pass (exact fast form, IEEE redo when flagged).
__device__ void pair_electrostatic_lds(const wg_batch &b, const KParams &kp, const float *spos, int lm, int M, int q,
                                       size_t g0, double md, double ym, float &ax, float &ay, float &az) {
    const float *p3 = spos + 3 * (lm + q);
    const double sq = b.charge ? b.charge[g0 + q] : kp.pair_e;
    const float sx = ax, sy = ay, sz = az;
    bool bad = false;
    {
        for (int pj = 0; pj < M; pj++) {
            if (pj == q) continue;
            const float *o3 = spos + 3 * (lm + pj);
            const double os = b.charge ? b.charge[g0 + pj] : kp.pair_e;
            pair_central_fast(kp.pair_k, sq, os, o3[0] - p3[0], o3[1] - p3[1], o3[2] - p3[2], md, ym, ax, ay, az, bad);
        }
        bad = bad || !__builtin_isfinite(ax + ay + az);
    }
    if (__builtin_expect(bad, 0)) {
        ax = sx; ay = sy; az = sz;
        for (int pj = 0; pj < M; pj++) {
            if (pj == q) continue;
            const float *o3 = spos + 3 * (lm + pj);
            const double os = b.charge ? b.charge[g0 + pj] : kp.pair_e;
            pair_central_term(kp.pair_k, sq, os, o3[0] - p3[0], o3[1] - p3[1], o3[2] - p3[2], md, ym, ax, ay, az);
        }
    }
}

// Mass q of the walker whose masses are LDS [lm, lm + M) and global [g0, g0 + M).
// One central-force pass of the workgroup kernel (GRAV: Point.gravity with s = m from LDS; else Point.coulomb with s
// = the charge): mass q meets its partners in ascending index, the strengths in the reference pair's (i < j) order.
template <bool GRAV>
__device__ __forceinline__ void pair_central_pass_lds(const wg_batch &b, double coef, double sq, const float *spos,
                                                      const float *sm, int lm, int M, int q, size_t g0, double pe,
                                                      double md, double ym, const float *p3, float &ax, float &ay,
                                                      float &az) {
    auto strength = [&](int pj) -> double {
        return GRAV ? (double)sm[lm + pj] : (b.charge ? (double)b.charge[g0 + pj] : pe);
    };
    const float sx = ax, sy = ay, sz = az;
    bool bad = false;
    if (M > 0) {
        const float *o3 = spos + 3 * lm;
        float n0 = o3[0], n1 = o3[1], n2 = o3[2];
        double ns = strength(0);
        for (int pj = 0; pj < M; pj++) {
            const float c0 = n0, c1 = n1, c2 = n2;
            const double os = ns;
            const int nx = min(pj + 1, M - 1);                  // (the last read repeats partner M - 1, unused)
            n0 = o3[3 * nx]; n1 = o3[3 * nx + 1]; n2 = o3[3 * nx + 2];
            ns = strength(nx);
            if (pj == q) continue;
            pair_central_fast(coef, pj < q ? os : sq, pj < q ? sq : os, c0 - p3[0], c1 - p3[1], c2 - p3[2], md, ym,
                              ax, ay, az, bad);
        }
        bad = bad || !__builtin_isfinite(ax + ay + az);
    }
    if (__builtin_expect(bad, 0)) {   // the exact pass: IEEE divisions and sqrtf
        ax = sx; ay = sy; az = sz;
        for (int pj = 0; pj < M; pj++) {
            if (pj == q) continue;
            const float *o3 = spos + 3 * (lm + pj);
            const double os = strength(pj);
            pair_central_term(coef, pj < q ? os : sq, pj < q ? sq : os, o3[0] - p3[0], o3[1] - p3[1], o3[2] - p3[2],
                              md, ym, ax, ay, az);
        }
    }
}

__device__ void pair_forces_lds(const wg_batch &b, const KParams &kp, const float *spos, const float *sm, int lm,
                                int M, int q, size_t g0, float mf, float &ax, float &ay, float &az) {
    const float *p3 = spos + 3 * (lm + q);
    const double md = (double)mf;
    const double ym = 1.0 / md;                  // every "/ m" below: ddiv_f32d (m is a float32 value)
    // gym/engine.py:128-137 (Config.g, m) and :139-147 (Config.k, e): one loop per pass, each partner's state read one
    // partner ahead (the term of partner pj computes while pj + 1's position and strength are in flight)
    if (kp.pair_mode & 1)
        pair_central_pass_lds<true>(b, kp.pair_g, md, spos, sm, lm, M, q, g0, 0.0, md, ym, p3, ax, ay, az);
    if (kp.pair_mode & 2)
        pair_central_pass_lds<false>(b, kp.pair_k, b.charge ? (double)b.charge[g0 + q] : kp.pair_e, spos, sm, lm, M, q,
                                     g0, kp.pair_e, md, ym, p3, ax, ay, az);
    if (kp.pair_mode & 4) {                  // gym/engine.py:114-125, partners j < q, then j != q, then j > q
        const double rs = b.radius[g0 + q];
        // bounce_set: bit 0 calls bounce, bit 1 is in `other` (pair_bounce, lean kernel); NULL = every point both
        const int bs = b.bounce_set ? (int)b.bounce_set[g0 + q] : 3;
        for (int ph = 0; ph < 3; ph++) {
            for (int pj = 0; pj < M; pj++) {
                const int obs = b.bounce_set ? (int)b.bounce_set[g0 + pj] : 3;
                const bool on = ph == 1 ? pj != q && (bs & 1) && (obs & 2)
                                        : (ph == 0 ? pj < q : pj > q) && (obs & 1) && (bs & 2);
                if (!on) continue;
                const float *o3 = spos + 3 * (lm + pj);
                const float d0 = o3[0] - p3[0], d1 = o3[1] - p3[1], d2 = o3[2] - p3[2];
                const float cur = np_norm3(d0, d1, d2);
                const double x = rs + b.radius[g0 + pj];
                if (!((double)cur <= x)) continue;
                const float dx = cur - (float)x;                                  // engine.py:96
                const float nf = -((-dx) * kp.bounce_kh);                         // -f_size, :75,100
                bounce_term(cur, nf, d0, d1, d2, md, ym, ax, ay, az);
            }
        }
    }
    if ((kp.pair_mode & 8) && M >= 2) {      // G2 Point.gravity: every a zeroed first (optimized_engine.py:174-175)
        ax = 0.f; ay = 0.f; az = 0.f;
        for (int pj = 0; pj < M; pj++) {
            if (pj == q) continue;
            const float *o3 = spos + 3 * (lm + pj);
            const double mo = (double)sm[lm + pj];
            g2_gravity_term<true>(((-kp.pair_g) * (pj < q ? mo : md)) * (pj < q ? md : mo), o3[0] - p3[0],
                                  o3[1] - p3[1], o3[2] - p3[2], mf, ym, ax, ay, az);
        }
    }
    if (kp.pair_mode & 16)                   // Point.electrostatic (gym/engine.py:150-158) of every point
        pair_electrostatic_lds(b, kp, spos, lm, M, q, g0, md, ym, ax, ay, az);
}

// ------------------------------------------------------------------ the step kernel
// STEP = false: observe only (reset path).  RAGGED: CSR offsets + block plan.  IN3D: obs layout.
// PWD: pairwise-sum recursion depth (0: M <= 128).  SHFL: register reductions (uniform, M | 64).
// Register budget of the step instances with the unrolled-once pairwise tree (PWD 0, no lane shuffles): 6 waves per
// SIMD, i.e. 80 VGPRs, so three 512-thread workgroups share a CU instead of two (the compiler's own choice, 90 VGPRs,
// is 5 waves per SIMD, which a 512-thread workgroup rounds down to 4): 4,096 chains of 100 masses 159.6 -> 153.8 us
// per launch, the performance_demo loop 181.9 -> 173.4 (profiles/r03v_ab_wg_occupancy.json); 7 spills more and
// gains less.  The PWD 3 and shuffle instances would spill 48-116 B at 80 VGPRs and keep the compiler's choice.
template <bool STEP, bool RAGGED, bool IN3D, int PWD, bool SHFL>
constexpr int wg_kernel_waves() { return (STEP && PWD == 0 && !SHFL) ? 6 : 1; }
template <bool STEP, bool RAGGED, bool IN3D, int PWD, bool SHFL>
__global__ __launch_bounds__(MAXT) __attribute__((amdgpu_waves_per_eu(wg_kernel_waves<STEP, RAGGED, IN3D, PWD, SHFL>()))) void walker_step_kernel(
    wg_batch b, KParams kp, const float *__restrict__ action, int action_cols, int action_stride,
    KOut o, const int32_t *__restrict__ plan, Geo geo) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    Carve s = carve(smem, geo);
    const int tid = threadIdx.x, lane = tid & 63, T = blockDim.x;

    // ---- this workgroup's walker range and flat slices
    int w0, w1;
    if (RAGGED) { w0 = plan[blockIdx.x]; w1 = plan[blockIdx.x + 1]; }
    else { w0 = blockIdx.x * geo.W; w1 = min(w0 + geo.W, b.N); }
    const int nw = w1 - w0;
    int P0, P1, E0, E1, U0, U1;
    if (RAGGED) {
        P0 = b.mass_off[w0]; P1 = b.mass_off[w1];
        E0 = b.edge_off[w0]; E1 = b.edge_off[w1];
        U0 = b.muscle_off[w0]; U1 = b.muscle_off[w1];
        for (int i = tid; i <= nw; i += T) {
            s.moff[i] = b.mass_off[w0 + i] - P0;
            s.eoff[i] = b.edge_off[w0 + i] - E0;
            s.uoff[i] = b.muscle_off[w0 + i] - U0;
        }
    } else {
        P0 = w0 * b.M; P1 = w1 * b.M; E0 = w0 * b.K; E1 = w1 * b.K; U0 = w0 * b.A; U1 = w1 * b.A;
    }
    const int nP = P1 - P0, nE = E1 - E0, nU = U1 - U0;

    // ================= phase 0: issue every global load of the tile =================
    stage_in<float4>(s.pos, b.pos + 3 * (size_t)P0, 3 * nP, tid, T);
    stage_in<float4>(s.vel, b.vel + 3 * (size_t)P0, 3 * nP, tid, T);
    if (!STEP && !SHFL) stage_in<float4>(s.acc, b.acc + 3 * (size_t)P0, 3 * nP, tid, T);
    if (!SHFL) stage_in<float4>(s.m, b.mass + P0, nP, tid, T);
    if (STEP && nE > 0)
        stage_in<uint4>(s.inc, reinterpret_cast<const uint32_t *>(b.inc) + E0, nE, tid, T);

    // edge records of this lane's first pass -> registers
    EdgeRec er[EPL];
    if (STEP) {
#pragma unroll
        for (int it = 0; it < EPL; it++) {
            const int le = tid + it * T;
            if (le < nE) er[it] = load_edge(b.edges, E0 + le);
        }
    }
    // muscles of this lane (first pass) -> registers
    float mu_x = 0.f, mu_lo = 0.f, mu_hi = 0.f, mu_st = 0.f, mu_a = 0.f;
    int mu_ua = 0, mu_wl = 0;
    if (tid < nU) {
        if (!RAGGED) { mu_wl = fdiv(tid, b.A, geo.invA); mu_ua = tid - mu_wl * b.A; }
        mu_x = b.muscle_x[U0 + tid];
        if (STEP && action) {
            const float2 bd = reinterpret_cast<const float2 *>(b.muscle_bounds)[U0 + tid];
            mu_lo = bd.x; mu_hi = bd.y;
            if (kp.action_mode == 1) mu_st = b.muscle_stride[U0 + tid];
            if (!RAGGED && mu_ua < action_cols) mu_a = action[(size_t)(w0 + mu_wl) * action_stride + mu_ua];
        }
    }
    // this lane's mass (first pass): walker, mass, incidence offsets, step counter
    int my_wl = 0, my_lm = 0;
    if (!RAGGED && tid < nP) { my_wl = fdiv(tid, b.M, geo.invM); my_lm = my_wl * b.M; }
    float my_m = 0.f;
    int wsteps = 0;
    if (SHFL) {
        if (tid < nP) {
            my_m = b.mass[P0 + tid];
            if (tid == my_lm) wsteps = b.steps[w0 + my_wl];
        }
    } else if (tid < nw) {
        wsteps = b.steps[w0 + tid];
    }
    if (RAGGED) {
        __syncthreads();   // walker offsets visible before lanes locate their walker
        if (tid < nP) { my_wl = locate(s.moff, nw, tid); my_lm = s.moff[my_wl]; }
    }
    int io0 = 0, io1 = 0;
    if (STEP && tid < nP) {
        const uint16_t *io = b.inc_off + (size_t)(P0 + my_lm) + (size_t)(w0 + my_wl);
        io0 = io[tid - my_lm];
        io1 = io[tid - my_lm + 1];
    }

    // ================= 1. act: Creature.act -> Muscle.act / actdisp -> regulation =================
    // (gym/optimized_walker.py:27-43,164-172)
    for (int u = tid; u < nU; u += T) {
        const bool first = (u == tid);
        float x = first ? mu_x : b.muscle_x[U0 + u];
        if (STEP && action) {
            int wl, ua;
            if (RAGGED) { wl = locate(s.uoff, nw, u); ua = u - s.uoff[wl]; }
            else if (first) { wl = mu_wl; ua = mu_ua; }
            else { wl = fdiv(u, b.A, geo.invA); ua = u - wl * b.A; }
            if (ua < action_cols) {
                float lo = mu_lo, hi = mu_hi, st = mu_st, a = mu_a;
                if (!first || RAGGED) {
                    if (!first) {
                        const float2 bd = reinterpret_cast<const float2 *>(b.muscle_bounds)[U0 + u];
                        lo = bd.x; hi = bd.y;
                        if (kp.action_mode == 1) st = b.muscle_stride[U0 + u];
                    }
                    a = action[(size_t)caller_row(b, w0 + wl) * action_stride + ua];
                }
                if (kp.action_mode == 1) x = (a != 0.f) ? x + st : x - st;
                else x = x + a;
                if (lo > x) x = lo;     // Python max(x, originx*minl)
                if (hi < x) x = hi;     // Python min(x, originx*maxl)
                b.muscle_x[U0 + u] = x;
            }
        }
        s.x[u] = x;
    }
    pw_tables_to_lds(tid);   // (np_sq_t's cold path: the pair passes, the energy terms)
    __syncthreads();

    // registers of this lane's (first) mass after the physics: feed the SHFL reductions and obs
    float px = 0.f, py = 0.f, pz = 0.f, vx = 0.f, vy = 0.f, vz = 0.f, ax = 0.f, ay = 0.f, az = 0.f;
    float nv = 0.f, ke = 0.f, pe = 0.f;
    if (STEP) {
        // ================= 2. edge phase =================
        // spring (gym/engine.py:78-102) + damping (gym/optimized_walker.py:92-106)
        bool gtiny = false;
        for (int pass = 0; pass * EPL * T < nE; pass++) {
#pragma unroll
            for (int it = 0; it < EPL; it++) {
                const int le = tid + (pass * EPL + it) * T;
                if (le >= nE) continue;   // (not break: an early exit kept er[] on the stack)
                const EdgeRec e = (pass == 0) ? er[it] : load_edge(b.edges, E0 + le);
                if (WG_ABLATE & 1) {
                    s.t[3 * le] = e.rest; s.t[3 * le + 1] = e.k; s.t[3 * le + 2] = e.c;
                    s.df[3 * le] = (float)(e.ij & 0xffu); s.df[3 * le + 1] = 0.f; s.df[3 * le + 2] = 0.f;
                    continue;
                }
                int lm, ew, Aw, ub;
                if (RAGGED) {
                    const int wl = locate(s.eoff, nw, le);
                    lm = s.moff[wl]; ew = le - s.eoff[wl]; Aw = s.uoff[wl + 1] - s.uoff[wl]; ub = s.uoff[wl];
                } else {
                    const int wl = fdiv(le, b.K, geo.invK);
                    lm = wl * b.M; ew = le - wl * b.K; Aw = b.A; ub = wl * b.A;
                }
                spring_edge(e, le, lm, (ew < Aw) ? s.x[ub + ew] : e.rest, s.pos, s.vel, s.t, s.df, kp.spring_mode,
                            gtiny);
            }
        }
        // any damping force of the tile outside the exact range of the mass loop's float32 quotient: IEEE divisions
        const bool tiny_blk = __syncthreads_or(gtiny) != 0;

        // ================= 3. mass phase: ordered accumulation, env forces, run1 =================
        const uint16_t *s_inc16 = reinterpret_cast<const uint16_t *>(s.inc);
        // mass lp's walker, its first mass and incidence range
        auto mass_of = [&](int lp, int &wl, int &lm, int &s0, int &s1) {
            const bool first = (lp == tid);
            if (first) { wl = my_wl; lm = my_lm; }
            else if (RAGGED) { wl = locate(s.moff, nw, lp); lm = s.moff[wl]; }
            else { wl = fdiv(lp, b.M, geo.invM); lm = wl * b.M; }
            s0 = io0; s1 = io1;
            if (!first) {
                const uint16_t *io = b.inc_off + (size_t)(P0 + lm) + (size_t)(w0 + wl);
                s0 = io[lp - lm]; s1 = io[lp - lm + 1];
            }
        };
        const bool pairs = !SHFL && kp.pair_mode != 0;   // block-uniform
        if (pairs) {
            // pair passes read the other masses' positions: every mass accumulates its springs
            // and pair terms first (into s.acc), the env forces and the integrator follow after a barrier
            for (int lp = tid; lp < nP; lp += T) {
                int wl, lm, s0, s1;
                mass_of(lp, wl, lm, s0, s1);
                const int lb = RAGGED ? s.eoff[wl] : wl * b.K;
                const int M = RAGGED ? s.moff[wl + 1] - lm : b.M;
                const float mf = s.m[lp];
                mass_accumulate(TermsAoS{s.t, s.df}, s_inc16 + 2 * lb, lb, s0, s1, mf, ax, ay, az, 0, tiny_blk);
                pair_forces_lds(b, kp, s.pos, s.m, lm, M, lp - lm, (size_t)P0 + lm, mf, ax, ay, az);
                s.acc[3 * lp] = ax; s.acc[3 * lp + 1] = ay; s.acc[3 * lp + 2] = az;
            }
            __syncthreads();
        }
        for (int lp = tid; lp < nP; lp += T) {
            int wl, lm, s0, s1;
            mass_of(lp, wl, lm, s0, s1);
            const int lb = RAGGED ? s.eoff[wl] : wl * b.K;
            const float mf = SHFL ? my_m : s.m[lp];
            const double md = (double)mf;
            bool hit;
            if (pairs) {
                ax = s.acc[3 * lp]; ay = s.acc[3 * lp + 1]; az = s.acc[3 * lp + 2];
                mass_tail(kp, mf, (float)(1.0 / md), s.pos + 3 * lp, s.vel + 3 * lp, px, py, pz, vx, vy, vz, ax, ay,
                          az, hit, b.pinned && b.pinned[P0 + lp]);
            } else {
                mass_step(kp, s.t, s.df, s_inc16 + 2 * lb, lb, s0, (WG_ABLATE & 2) ? min(s1, s0 + 1) : s1, mf,
                          s.pos + 3 * lp, s.vel + 3 * lp, px, py, pz, vx, vy, vz, ax, ay, az, hit, kp.spring_mode,
                          b.pinned && b.pinned[P0 + lp], tiny_blk);
            }
            if (b.contact) b.contact[P0 + lp] = (uint8_t)hit;
            if (b.radius) b.radius[P0 + lp] = hit ? 3.0 : 1.0;   // gym/optimized_env.py:156,175
            s.pos[3 * lp] = px; s.pos[3 * lp + 1] = py; s.pos[3 * lp + 2] = pz;
            s.vel[3 * lp] = vx; s.vel[3 * lp + 1] = vy; s.vel[3 * lp + 2] = vz;
            if (SHFL) {      // old_a straight from registers (no LDS copy in the register-reduction kernel)
                float *ga = b.acc + 3 * ((size_t)P0 + lp);
                ga[0] = ax; ga[1] = ay; ga[2] = az;
            } else {
                s.acc[3 * lp] = ax; s.acc[3 * lp + 1] = ay; s.acc[3 * lp + 2] = az;
            }
            // reduction terms of the new state: |v|, m*|v|^2, f32(m*g)*(y-ground)
            nv = np_norm3(vx, vy, vz);
            ke = mf * np_sq_t<true>(nv);   // p.m * norm(p.v) ** 2 (gym/optimized_env.py:242)
            pe = (float)(md * kp.g) * (py - kp.ground);
            if (!SHFL) { s.nrm[lp] = nv; s.ke[lp] = ke; s.pe[lp] = pe; }
        }
    } else {
        for (int lp = tid; lp < nP; lp += T) {
            const float mf = SHFL ? my_m : s.m[lp];
            vx = s.vel[3 * lp]; vy = s.vel[3 * lp + 1]; vz = s.vel[3 * lp + 2];
            px = s.pos[3 * lp]; py = s.pos[3 * lp + 1]; pz = s.pos[3 * lp + 2];
            if (SHFL) {
                const float *ga = b.acc + 3 * ((size_t)P0 + lp);
                ax = ga[0]; ay = ga[1]; az = ga[2];
            } else {
                ax = s.acc[3 * lp]; ay = s.acc[3 * lp + 1]; az = s.acc[3 * lp + 2];
            }
            nv = np_norm3(vx, vy, vz);
            ke = mf * np_sq_t<true>(nv);
            pe = (float)((double)mf * kp.g) * (py - kp.ground);
            if (!SHFL) { s.nrm[lp] = nv; s.ke[lp] = ke; s.pe[lp] = pe; }
        }
    }

    // ================= per-walker reductions + outputs (gym/optimized_env.py:189-248) =================
    float midx = 0.f, midy = 0.f, midz = 0.f;
    float sumx = 0.f, sumy = 0.f, sumz = 0.f;   // walker position sums (G1 getstat, midform 2)
    const bool is_mass = tid < nP;
    const int my_q = tid - my_lm;
    if (SHFL) {
        const int M = b.M;
        const int gbase = (tid & ~63) + ((lane / M) * M);
        float sx, sy, sz;
        seq_sum3_lanes(px, py, pz, gbase, M, sx, sy, sz);
        const float ysum = pw_sum_lanes(py, gbase, M, lane), vsum = pw_sum_lanes(nv, gbase, M, lane);
        const float ksum = pw_sum_lanes(ke, gbase, M, lane), psum = pw_sum_lanes(pe, gbase, M, lane);
        const unsigned long long gmask = (M == 64) ? ~0ull : (((1ull << M) - 1ull) << (gbase & 63));
        // the collision penalty counts contacts of the NEW state (optimized_env.py:200 runs after run1)
        const unsigned long long hb = __ballot(is_mass && (py - kp.ground < 0.f));
        const unsigned long long sb = __ballot(is_mass && nv < 0.1f);
        const int hits = __popcll(hb & gmask);
        const bool all_stopped = (sb & gmask) == gmask;
        const float fM = (float)M;
        midx = sx / fM; midy = sy / fM; midz = sz / fM;
        sumx = sx; sumy = sy; sumz = sz;
        if (is_mass && my_q == 0) {
            const size_t wg = (size_t)(w0 + my_wl);
            int steps = wsteps;
            if (STEP) { steps += 1; b.steps[wg] = steps; }
            if (o.steps) o.steps[wg] = steps;
            const float cy = ysum / fM;
            if (o.reward) {
                const float vpen = (-(vsum / fM)) * 0.1f;
                o.reward[wg] = (cy + vpen) + (float)(-(double)hits * 0.5);
            }
            if (o.done) {
                int done = steps >= kp.max_steps;
                if (!done && cy < kp.done_y) done = 1;
                if (!done && steps > 100) done = all_stopped;
                o.done[wg] = (uint8_t)done;
            }
            if (o.centroid) { o.centroid[3 * wg] = midx; o.centroid[3 * wg + 1] = midy; o.centroid[3 * wg + 2] = midz; }
            if (o.energy) o.energy[wg] = 0.5f * ksum + psum;
        }
    }
    __syncthreads();

    if (STEP) {
        stage_out(b.pos + 3 * (size_t)P0, s.pos, 3 * nP, tid, T);
        stage_out(b.vel + 3 * (size_t)P0, s.vel, 3 * nP, tid, T);
        if (!SHFL) stage_out(b.acc + 3 * (size_t)P0, s.acc, 3 * nP, tid, T);
    }
    if (!SHFL) {
        // 8 lanes per walker, numpy's summation orders (see oracle/walker_oracle.c walker_observe):
        // r 0-2 sequential sums of pos[:, r] (getstat mid / info centroid), r 3 pairwise sum of y
        // (np.mean), r 4-6 pairwise sums of |v|, m|v|^2, m*g*(y-ground), r 7 contact count + all-stopped.
        for (int idx = tid; idx < ((WG_ABLATE & 8) ? 0 : nw * 8); idx += T) {
            const int wl = idx >> 3, r = idx & 7;
            const int lm = RAGGED ? s.moff[wl] : wl * b.M;
            const int M = RAGGED ? s.moff[wl + 1] - lm : b.M;
            float v;
            if (r == 7) {
                int hits = 0, all = 1;
                for (int q = 0; q < M; q++) {
                    hits += (s.pos[3 * (lm + q) + 1] - kp.ground < 0.f);
                    all &= (s.nrm[lm + q] < 0.1f);
                }
                v = __int_as_float((hits << 1) | all);
            } else {
                const float *src = r < 3 ? s.pos + 3 * lm + r
                                 : r == 3 ? s.pos + 3 * lm + 1
                                 : r == 4 ? s.nrm + lm : r == 5 ? s.ke + lm : s.pe + lm;
                const int st = r <= 3 ? 3 : 1;
                if (r < 3) {
                    v = seq_sum_lds(0.f, src, M, st);
                } else {
                    v = np_pairwise<PWD>(src, M, st);
                }
            }
            s.red[idx] = v;
        }
        __syncthreads();
        if (tid < nw) {
            const int wl = tid;
            const int lm = RAGGED ? s.moff[wl] : wl * b.M;
            const int M = RAGGED ? s.moff[wl + 1] - lm : b.M;
            const size_t ws = (size_t)(w0 + wl);             // stored walker (steps)
            const size_t wg = (size_t)caller_row(b, w0 + wl);   // the caller's row (outputs)
            const float fM = (float)M;
            const float *rd = s.red + 8 * wl;
            const float cy = rd[3] / fM;
            const int packed = __float_as_int(rd[7]);
            const int hits = packed >> 1, all = packed & 1;
            int steps = wsteps;
            if (STEP) { steps += 1; b.steps[ws] = steps; }
            if (o.steps) o.steps[wg] = steps;
            if (o.reward) {
                const float av = rd[4] / fM;
                const float vpen = (-av) * 0.1f;
                const float cpen = (float)(-(double)hits * 0.5);
                o.reward[wg] = (cy + vpen) + cpen;
            }
            if (o.done) {
                int done = steps >= kp.max_steps;
                if (!done && cy < kp.done_y) done = 1;
                if (!done && steps > 100) done = all;
                o.done[wg] = (uint8_t)done;
            }
            if (o.centroid) {
                o.centroid[3 * wg] = rd[0] / fM; o.centroid[3 * wg + 1] = rd[1] / fM; o.centroid[3 * wg + 2] = rd[2] / fM;
            }
            if (o.energy) o.energy[wg] = 0.5f * rd[5] + rd[6];
        }
    }

    // ================= observation rows: Creature.getstat (gym/optimized_walker.py:129-162) =================
    if (o.obs && !(WG_ABLATE & 16)) {
        constexpr int d = IN3D ? 3 : 2, per = 3 * d;
        const int stride = o.obs_stride;
        float *ob = o.obs + (uint32_t)w0 * (uint32_t)stride;
        // uniform batches assemble the rows in LDS (aliasing the dead spring-term region) and stream
        // them out as one contiguous 16-B-store block; ragged batches write rows directly.
        float *tile = RAGGED ? nullptr : reinterpret_cast<float *>(s.t);
        const int nmid = kp.conmid ? 3 : 0;
        if (SHFL) {
            if (is_mass) {
                float *row = tile + (size_t)my_wl * stride + per * my_q;
                const float pm[3] = {px, py, pz}, vm[3] = {vx, vy, vz}, am[3] = {ax, ay, az};
                // G1 getstat (midform 2, gym/walker.py:88-96) subtracts the SUM of positions
                const float mm[3] = {kp.midform == 2 ? sumx : midx, kp.midform == 2 ? sumy : midy,
                                     kp.midform == 2 ? sumz : midz};
#pragma unroll
                for (int c = 0; c < d; c++) {
                    row[c] = kp.midform ? (pm[c] - mm[c]) * kp.pk : pm[c] * kp.pk;
                    row[d + c] = vm[c] * kp.vk;
                    row[2 * d + c] = am[c] * kp.ak;
                }
                if (my_q == 0 && nmid) {
                    float *wrow = tile + (size_t)my_wl * stride + per * b.M;
                    wrow[0] = kp.midform ? mm[0] : 0.f; wrow[1] = kp.midform ? mm[1] : 0.f; wrow[2] = kp.midform ? mm[2] : 0.f;
                }
                if (my_q == 0)
                    for (int r = per * b.M + nmid + b.A; r < stride; r++) tile[(size_t)my_wl * stride + r] = 0.f;
            }
        } else {
            // per-mass block of 3*d values: (pos - mid)*pk, v*vk, old_a*ak
            for (int lp = tid; lp < nP; lp += T) {
                int wl, lm;
                if (lp == tid) { wl = my_wl; lm = my_lm; }
                else if (RAGGED) { wl = locate(s.moff, nw, lp); lm = s.moff[wl]; }
                else { wl = fdiv(lp, b.M, geo.invM); lm = wl * b.M; }
                const int M = RAGGED ? s.moff[wl + 1] - lm : b.M;
                const float fM = (float)M;
                float *row = (RAGGED ? o.obs + (size_t)caller_row(b, w0 + wl) * stride : tile + (size_t)wl * stride) +
                             per * (lp - lm);
#pragma unroll
                for (int c = 0; c < d; c++) {
                    const float pv = s.pos[3 * lp + c];
                    const float mid = kp.midform == 2 ? s.red[8 * wl + c] : s.red[8 * wl + c] / fM;   // G1: the sum
                    row[c] = kp.midform ? (pv - mid) * kp.pk : pv * kp.pk;
                    row[d + c] = s.vel[3 * lp + c] * kp.vk;
                    row[2 * d + c] = s.acc[3 * lp + c] * kp.ak;
                }
            }
            // conmid columns and zero padding of short (ragged) rows
            for (int wl = tid; wl < nw; wl += T) {
                const int lm = RAGGED ? s.moff[wl] : wl * b.M;
                const int M = RAGGED ? s.moff[wl + 1] - lm : b.M;
                const int A = RAGGED ? s.uoff[wl + 1] - s.uoff[wl] : b.A;
                float *row = RAGGED ? o.obs + (size_t)caller_row(b, w0 + wl) * stride : tile + (size_t)wl * stride;
                if (nmid)
                    for (int c = 0; c < 3; c++)
                        row[per * M + c] = kp.midform == 2 ? s.red[8 * wl + c] : kp.midform ? s.red[8 * wl + c] / (float)M : 0.f;
                for (int r = per * M + nmid + A; r < stride; r++) row[r] = 0.f;
            }
        }
        // muscle rest lengths x*mk
        for (int u = tid; u < nU; u += T) {
            int wl, ua, M;
            if (RAGGED) { wl = locate(s.uoff, nw, u); ua = u - s.uoff[wl]; M = s.moff[wl + 1] - s.moff[wl]; }
            else { wl = fdiv(u, b.A, geo.invA); ua = u - wl * b.A; M = b.M; }
            (RAGGED ? o.obs + (size_t)caller_row(b, w0 + wl) * stride : tile + (size_t)wl * stride)[per * M + nmid + ua] =
                s.x[u] * kp.mk;
        }
        if (!RAGGED) {
            __syncthreads();
            stage_out(ob, tile, nw * stride, tid, T);
        }
    }
}


// ------------------------------------------------------------------ lean wave-independent kernel
// Uniform batches with M | 64 (4 <= M <= 64): one mass per lane, 64/M walkers per wave and NO
// workgroup barrier.  Each wave owns a private LDS slice and runs its own load -> act -> springs ->
// masses -> outputs sequence, so the four waves of a workgroup (and the workgroups sharing a CU) drift
// apart and overlap one another's memory and compute phases instead of meeting at __syncthreads
// (the phase lock measured on walker_step_kernel).  Same arithmetic as
// walker_step_kernel, op for op; the only change is the spring's 1/dist (see rcp64_nr).
struct LeanGeo {
    int wpw;                                  // walkers per wave (64 / M)
    int wpb;                                  // waves per workgroup
    int lgM;                                  // log2(M)
    int slice;                                // LDS bytes per wave
    int off_df, off_inc, off_x;               // byte offsets in the slice (spring terms at 0)
    int pl;                                   // spring-term slots of a wave tile (>= wpw * K, multiple of 4)
    float invK, invA, invM;                   // invM = 1/M, exact (M | 64 is a power of two)
    int nblk;                                 // the launch's workgroup count (xcd_block), an explicit argument: read
                                              // from the dispatch packet it costs a dependent scalar round
};

// LDS hand-off between lanes of ONE wave: a wave's LDS operations execute in order, so a compiler
// barrier (wavefront-scope fences around the wave barrier) is all the ordering needed.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}


// Gather a float from another lane of the wave (ds_bpermute: LDS crossbar, no LDS allocation).  Executed
// by every lane (convergent): a lane that is inactive as a SOURCE would read back as 0.
__device__ __forceinline__ float lane_gather(float v, int src_byte) {
    return __int_as_float(__builtin_amdgcn_ds_bpermute(src_byte, __float_as_int(v)));
}

// Spring term and damping force of one edge from its endpoints' state (gathered from the mass lanes):
// spring_edge's arithmetic with the cheaper reciprocal (identical results; cold path unchanged).
// Cold path: every quantity again with IEEE divisions and numpy's sqrt (exact for every input).
__device__ __forceinline__ void spring_terms_cold(const EdgeRec &e, float x, float r0, float r1, float r2, double &t0,
                                               double &t1, double &t2, float &d0, float &d1, float &d2,
                                               int spring_mode) {
    const float cur = np_norm3(-r0, -r1, -r2);                      // engine.py:86 (p_i - p_j)
    const float dx = cur - x;                                       // engine.py:96
    double dist = (double)cur;                                      // engine.py:73
    if (CONFIG_R > dist) dist = CONFIG_R;                           // Python max(distance, r), NaN kept
    const float fsz = (spring_mode == 1 || !(dx < 0.f && edge_string(e.ij))) ? (-dx) * e.k : 0.f;  // :97-100
    const float nf = -fsz;                                                                           // :75
    d0 = r0; d1 = r1; d2 = r2;
    if (cur > 0.f) { d0 = r0 / cur; d1 = r1 / cur; d2 = r2 / cur; }
    if (spring_mode == 1) {
        t0 = (double)(fsz * d0); t1 = (double)(fsz * d1); t2 = (double)(fsz * d2);
    } else {
        t0 = (double)(nf * r0) / dist; t1 = (double)(nf * r1) / dist; t2 = (double)(nf * r2) / dist;
    }
}


// pos_ok (wave-uniform): every position component of the wave's masses is 0 or at least 2^-56 in magnitude, so every
// difference r is 0 or at least 2^-79 (a multiple of 2^-79, the spacing of floats at 2^-56) and the d quotients' dividends
// are in the exact range without a test per spring
__device__ __forceinline__ void spring_terms(const EdgeRec &e, float x, float pix, float piy, float piz, float pjx,
                                             float pjy, float pjz, float vix, float viy, float viz, float vjx,
                                             float vjy, float vjz, double &t0, double &t1, double &t2, float &g0,
                                             float &g1, float &g2, int spring_mode, bool pos_ok) {
    const float r0 = pjx - pix, r1 = pjy - piy, r2 = pjz - piz;     // other.pos - self.pos
    float d0, d1, d2;
    // np.linalg.norm(p_i - p_j) (engine.py:86): squares summed in float64, rounded, sqrt.  (p_i - p_j)^2 == r^2.
    const float sq = (float)(((double)(r0 * r0) + (double)(r1 * r1)) + (double)(r2 * r2));
    // sqrt_mid's range is [2^-96, 2^126); the d quotients' exact range asks cur in [2^-20, 2^20) (false for NaN)
    const bool mid = sq >= 0x1p-40f && sq < 0x1p40f;
    const float cur = sqrt_mid(sq);
    const float dx = cur - x;                                       // engine.py:96
    // cur >= 2^-48 > Config.r: max(distance, r) is the distance itself
    const double dist = (double)cur;
    const double yc = rcp64_nr(dist);
    const float fsz = (spring_mode == 1 || !(dx < 0.f && edge_string(e.ij))) ? (-dx) * e.k : 0.f;  // :97-100
    const float nf = -fsz;                                                                           // :75
    const float ycf = (float)yc;
    d0 = fdiv_fast(r0, cur, ycf); d1 = fdiv_fast(r1, cur, ycf); d2 = fdiv_fast(r2, cur, ycf);
    if (spring_mode == 1) {
        t0 = (double)(fsz * d0); t1 = (double)(fsz * d1); t2 = (double)(fsz * d2);
    } else {
        t0 = ddiv_fast((double)(nf * r0), dist, yc);
        t1 = ddiv_fast((double)(nf * r1), dist, yc);
        t2 = ddiv_fast((double)(nf * r2), dist, yc);
    }
    bool rok = true;
    if (__builtin_expect(!pos_ok, 0)) rok = fexp3(r0, r1, r2) >= TINY_EXP;
    // mid holds only for finite differences with |r| < 2^20 (an inf / NaN / overflowing square fails it), so the d
    // quotients are finite; |nf| < 2^100 (false for NaN) keeps nf * r below 2^120 and every t quotient finite and in
    // Markstein's exact range (|t| in [2^-170, 2^140] or 0): the same lanes' quotients as the finiteness tests of
    // d and t certified, with five fewer VALU (a larger |nf| now takes the exact cold path too: same results)
    const bool fast_ok = mid && rok && __builtin_fabsf(nf) < 0x1p100f;
    if (__builtin_expect(!fast_ok, 0)) spring_terms_cold(e, x, r0, r1, r2, t0, t1, t2, d0, d1, d2, spring_mode);
    const float dk = np_dot3(vix - vjx, viy - vjy, viz - vjz, d0, d1, d2);  // optimized_walker.py:102-103
    const float dkc = dk * e.c;                                               // :104
    g0 = dkc * d0; g1 = dkc * d1; g2 = dkc * d2;
}
// gt: a damping-force component below the exact range of the mass loop's float32 quotient (the wave then runs its mass
// loop with IEEE divisions)
template <class TS>
__device__ __forceinline__ void spring_edge_regs(const EdgeRec &e, int le, float x, float pix, float piy, float piz,
                                                 float pjx, float pjy, float pjz, float vix, float viy, float viz,
                                                 float vjx, float vjy, float vjz, const TS &ts, int spring_mode, bool &gt,
                                                 bool pos_ok) {
    double t0, t1, t2;
    float g0, g1, g2;
    spring_terms(e, x, pix, piy, piz, pjx, pjy, pjz, vix, viy, viz, vjx, vjy, vjz, t0, t1, t2, g0, g1, g2, spring_mode,
                 pos_ok);
    ts.put(le, t0, t1, t2, g0, g1, g2);
    gt = gt || fexp3(g0, g1, g2) < TINY_EXP;
}

// ------------------------------------------------------------------ lean wave tile: loads, then compute
// Global inputs of one wave's tile, held in registers: lean_load issues every HBM read of the tile back to
// back, lean_compute consumes them.
template <int NE>
struct LeanIn {
    float p3[3], v3[3];          // this lane's mass: pos, vel (the springs gather them with ds_bpermute)
    EdgeRec er[NE];              // this lane's spring record in each edge pass
    uint32_t gi[NE];             // incidence words (two u16 entries each)
    float mf;                    // mass
    int io0, io1, wsteps, pin;   // incidence range; step counter (q == 0 lanes); DingPoint flag
    float x, lo, hi, stp, a;     // this lane's muscle: Muscle.x, regulation bounds, stride, action
};

// A wave's tile: its walker range and the lane roles in it (no memory access).
struct LeanTile {
    int w0, nw, nP, nE, nU, wl, q, mu_wl, mu_ua;
    uint32_t P0, E0, U0;         // 32-bit element offsets (host-checked to fit)
    bool is_mass, is_mus, acts;
};

__device__ __forceinline__ LeanTile lean_tile_of(const wg_batch &b, const float *action, int action_cols,
                                                 const LeanGeo &lg, int tile, int lane) {
    LeanTile t;
    t.w0 = tile * lg.wpw;
    t.nw = min(lg.wpw, b.N - t.w0);
    t.nP = t.nw * b.M; t.nE = t.nw * b.K; t.nU = t.nw * b.A;
    t.P0 = (uint32_t)t.w0 * b.M; t.E0 = (uint32_t)t.w0 * b.K; t.U0 = (uint32_t)t.w0 * b.A;
    t.wl = lane >> lg.lgM; t.q = lane & (b.M - 1);
    t.is_mass = lane < t.nP;
    t.is_mus = lane < t.nU;
    t.mu_wl = b.A > 0 ? fdiv(lane, b.A, lg.invA) : 0;
    t.mu_ua = lane - t.mu_wl * b.A;
    t.acts = action != nullptr && t.is_mus && t.mu_ua < action_cols;
    return t;
}

// Every global load of the wave's walkers, issued back to back: pos, vel, spring records with their incidence
// words, mass-loop inputs, muscles.  (Issuing what the springs need first and the mass-loop inputs last measured
// 48.5 against 47.7 us per launch, profiles/r02_ab_loadorder_karg.json: in steady state a wave spends ~4K of its
// ~25K cycles on loads, so there is little latency left to hide.)
// A global array element at a 32-bit byte offset from a kernel-argument base: the address is SGPR base + zero-extended
// VGPR offset, which the global_load's saddr form takes as is (no 64-bit address arithmetic per load).
template <typename T>
__device__ __forceinline__ const T &at_u32(const T *base, uint32_t byte_off) {
    return *reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) + (size_t)byte_off);
}
// The same form for the stores (global_store's saddr form): the lean and wave kernels' outputs, whose byte offsets the
// host bounds below 4 GiB (u32_bytes, obs_u32).
template <typename T>
__device__ __forceinline__ T &at_u32w(T *base, uint32_t byte_off) {
    return *reinterpret_cast<T *>(reinterpret_cast<char *>(base) + (size_t)byte_off);
}
// a walker's (or mass's) element e of a record of n floats, as a 32-bit byte offset
#define WG_ST(base, e, n) (&at_u32w((base), (uint32_t)(n) * 4u * (uint32_t)(e)))
// a count (<= 64) halved and negated as the reference's float64 product: exact in float32 (-0.0 for 0, as -(0.0) * 0.5)
__device__ __forceinline__ float neg_half_count(int n) { return -0.5f * (float)n; }
template <int NE>
__device__ __forceinline__ void lean_load_mass(const wg_batch &b, const LeanTile &t, int lane, LeanIn<NE> &L) {
    L.mf = 0.f; L.io0 = 0; L.io1 = 0; L.wsteps = 0; L.pin = 0;
    // every lane loads (lanes past the tile's masses a duplicate of its last one; their values are never used)
    const int ln = min(lane, t.nP - 1);
    const int wl = ln >> (31 - __builtin_clz(b.M)), q = ln & (b.M - 1);
    L.mf = at_u32(b.mass, 4u * (t.P0 + ln));
    if (b.pinned) L.pin = at_u32(b.pinned, t.P0 + ln);
    const uint32_t io = (uint32_t)(t.w0 + wl) * (b.M + 1) + q;
    L.io0 = at_u32(b.inc_off, 2u * io); L.io1 = at_u32(b.inc_off, 2u * io + 2u);
    L.wsteps = at_u32(b.steps, 4u * (uint32_t)(t.w0 + wl));   // the walker's counter in each of its lanes
}
template <int NE>
__device__ __forceinline__ void lean_load_muscles(const wg_batch &b, const KParams &kp, const float *__restrict__ action,
                                                  int action_stride, const LeanTile &t, int lane, LeanIn<NE> &L) {
    L.x = 0.f; L.lo = 0.f; L.hi = 0.f; L.stp = 0.f; L.a = 0.f;
    if (t.nU > 0) {                       // wave-uniform
        const uint32_t ul = t.U0 + min(lane, t.nU - 1);
        L.x = at_u32(b.muscle_x, 4u * ul);
        if (action && action_stride > 0) {
            const float2 bd = at_u32(reinterpret_cast<const float2 *>(b.muscle_bounds), 8u * ul);
            L.lo = bd.x; L.hi = bd.y;
            if (kp.action_mode == 1) L.stp = at_u32(b.muscle_stride, 4u * ul);
            const int wl = min(t.mu_wl, t.nw - 1), ua = max(0, min(t.mu_ua, action_stride - 1));
            L.a = at_u32(action, 4u * ((uint32_t)(t.w0 + wl) * (uint32_t)action_stride + (uint32_t)ua));
        }
    }
}
template <int NE>
__device__ __forceinline__ void lean_load(const wg_batch &b, const KParams &kp, const float *__restrict__ action,
                                          int action_stride, const LeanTile &t, int lane, LeanIn<NE> &L) {
    // every load unconditional from a clamped (valid) index, issued back to back: no exec-mask branch per load
    // (each with its zero-fill moves), addresses as SGPR base + 32-bit offset.  Lanes past the tile's masses,
    // springs and muscles hold duplicates; every use of them is gated (is_mass, le < nE, is_mus, acts).
    const uint32_t pl = t.P0 + min(lane, t.nP - 1);
    const float *gp = &at_u32(b.pos, 12u * pl), *gv = &at_u32(b.vel, 12u * pl);
    L.p3[0] = gp[0]; L.p3[1] = gp[1]; L.p3[2] = gp[2];
    L.v3[0] = gv[0]; L.v3[1] = gv[1]; L.v3[2] = gv[2];
#pragma unroll
    for (int it = 0; it < NE; it++) {
        const uint32_t le = t.E0 + (uint32_t)min(lane + 64 * it, t.nE - 1);
        const uint4 v = at_u32(reinterpret_cast<const uint4 *>(b.edges), 16u * le);
        L.er[it] = EdgeRec{v.x, __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
        L.gi[it] = at_u32(reinterpret_cast<const uint32_t *>(b.inc), 4u * le);
    }
    lean_load_mass<NE>(b, t, lane, L);
    lean_load_muscles<NE>(b, kp, action, action_stride, t, lane, L);
    if (!t.is_mass) {                     // the reference values of the lanes past the tile's masses
        L.p3[0] = 0.f; L.p3[1] = 0.f; L.p3[2] = 0.f; L.v3[0] = 0.f; L.v3[1] = 0.f; L.v3[2] = 0.f;
        L.mf = 0.f; L.pin = 0; L.io0 = 0; L.io1 = 0;
    }
    if (!t.is_mus) { L.x = 0.f; L.lo = 0.f; L.hi = 0.f; L.stp = 0.f; }
    if (!t.acts) L.a = 0.f;
}

// double gathered from another lane (two ds_bpermute), all lanes taking part
__device__ __forceinline__ double lane_gather_d(double v, int src_byte) {
    return __hiloint2double(__builtin_amdgcn_ds_bpermute(src_byte, __double2hiint(v)),
                            __builtin_amdgcn_ds_bpermute(src_byte, __double2loint(v)));
}

// numpy's float32 x ** 2 for the latency-bound NE = 1 tiles with glibc's two tables held in the wave's registers (lane
// l < 32: log2 table entry l in tl, exp2 entry l in te) and read by ds_bpermute: the restated powf's two dependent
// table reads cost two LDS-crossbar round trips instead of two global-memory ones.  Convergent: every lane of the wave
// runs it (the caller branches on a ballot); pw_pow2's arithmetic and special cases, unchanged (powf2.h).  Checked on the
// GPU against pw_pow2 for every float32 bit pattern (scripts/check_pow2_lanes.hip, profiles/r04x_check_pow2_lanes.json);
// Balance-4096 5.48 -> 5.37 us (the cold path, ~9 % of its waves, cost 0.28 us: RN(x*x) everywhere ran 5.20;
// profiles/r04x_ab_balance_sq.json).
__device__ __forceinline__ float pw_pow2_lanes(float x, double tl, double te) {
    unsigned int ix = pw_asu32(x) & 0x7fffffffu;
    const bool special = ix == 0u || ix >= 0x7f800000u;          // zero, inf, nan: glibc returns x * x
    if (ix < 0x00800000u && ix != 0u) {                          // subnormal: normalise (the product is exact)
        ix = pw_asu32(pw_asfloat(ix) * 0x1p23f) & 0x7fffffffu;
        ix -= 23u << 23;
    }
    const unsigned int tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) & 15u);
    const unsigned int top = tmp & 0xff800000u;
    const int k = (int)top >> 23;
    const double invc = lane_gather_d(tl, (2 * i) << 2), logc = lane_gather_d(tl, (2 * i + 1) << 2);
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
    const bool big = ((pw_asu64(xd) >> 47) & 0xffffu) >= (pw_asu64(126.0) >> 47);   // |2 log2 x| >= 126
    const double shift = 0x1.8p+47;
    double kd = xd + shift;
    const unsigned long long ki = pw_asu64(kd);
    kd -= shift;
    const double rr = xd - kd;
    const unsigned long long t = pw_asu64(lane_gather_d(te, (int)(ki & 31u) << 2)) + (ki << 47);
    const double sc = pw_asdouble(t);
    const double zz = PW_FMA(0x1.c6af84b912394p-5, rr, 0x1.ebfce50fac4f3p-3);
    const double rr2 = rr * rr;
    double yy = PW_FMA(0x1.62e42ff0c52d6p-1, rr, 1.0);
    yy = PW_FMA(zz, rr2, yy);
    float res = (float)(yy * sc);
    if (big && xd > 0x1.fffffffd1d571p+6) res = pw_asfloat(0x7f800000u);   // overflow: +inf
    else if (big && xd <= -150.0) res = 0.0f;                              // underflow: +0
    return special ? x * x : res;
}
// np_sq for every lane of the wave at once (called outside any per-lane branch): RN(x*x) where that is provably
// powf's value, the lane-table powf for the wave's lanes that need it
__device__ __forceinline__ float np_sq_wave(float x, double tl, double te) {
    float f;
    const bool need = !pw_pow2_fast(x, &f);
    if (__builtin_expect(__ballot(need) != 0ull, 0)) {
        const float g = pw_pow2_lanes(x, tl, te);
        if (need) f = g;
    }
    return f;
}

// pair_mode bits 1 / 2: Point.gravity / Point.coulomb (gym/engine.py:128-147) restricted to the walker's
// masses, after its springs.  Mass q meets its partners in the reference pair loop's order
// (i < j): ascending partner index.  Per partner: r = max(norm(p_i - p_j) as float64, Config.r);
// f = -c*s_i*s_j/r**2 in float64 (c, s = Config.g, m or Config.k, e; i the lower index); anti_forced (:69-76):
// force = (-f * (p_partner - p_q)) / r, all float64 (f is a numpy float64 scalar, r came from .astype(float));
// forced (:65-67): a = f32(f64(a) + force/m).  Every lane runs the loop (partner state by ds_bpermute);
// non-mass lanes discard theirs.  IEEE float64 divisions: an opt-in mode, not the headline path.
// self_first (Point.electrostatic, gym/engine.py:150-158): f = -Config.k * e_q * e_partner for every partner (self's
// charge first) instead of the lower index's first.
__device__ __forceinline__ void pair_central(double coef, double sq, const float *p3, float mf, int lane, int M,
                                             bool is_mass, float &ax, float &ay, float &az, bool self_first = false) {
    const int gb = lane & ~(M - 1), q = lane & (M - 1);
    const double md = (double)mf, ym = 1.0 / md;
    const float sx = ax, sy = ay, sz = az;
    bool bad = false;
    {
        for (int pj = 0; pj < M; pj++) {
            const int src = (gb + pj) << 2;
            const float ox = lane_gather(p3[0], src), oy = lane_gather(p3[1], src), oz = lane_gather(p3[2], src);
            const double os = lane_gather_d(sq, src);
            if (!is_mass || pj == q) continue;
            const float d0 = ox - p3[0], d1 = oy - p3[1], d2 = oz - p3[2];   // partner - self
            const bool lo = pj < q && !self_first;
            pair_central_fast(coef, lo ? os : sq, lo ? sq : os, d0, d1, d2, md, ym, ax, ay, az, bad);
        }
        bad = is_mass && (bad || !__builtin_isfinite(ax + ay + az));
    }
    // the exact pass (IEEE divisions and sqrtf) for the lanes that need it; every lane gathers (wave-uniform branch)
    if (__builtin_expect(__ballot(bad) != 0, 0)) {
        float cx = sx, cy = sy, cz = sz;
        for (int pj = 0; pj < M; pj++) {
            const int src = (gb + pj) << 2;
            const float ox = lane_gather(p3[0], src), oy = lane_gather(p3[1], src), oz = lane_gather(p3[2], src);
            const double os = lane_gather_d(sq, src);
            if (!bad || pj == q) continue;
            const float d0 = ox - p3[0], d1 = oy - p3[1], d2 = oz - p3[2];
            const bool lo = pj < q && !self_first;
            pair_central_term(coef, lo ? os : sq, lo ? sq : os, d0, d1, d2, md, ym, cx, cy, cz);
        }
        if (bad) { ax = cx; ay = cy; az = cz; }
    }
}

// pair_mode bit 4: Point.bounce(k) (gym/engine.py:114-125) for every point of the walker in registry order:
// for each other point i, if norm(s.pos - i.pos).astype(float) <= s.r + i.r, s.resilience(i, s.r + i.r, k/2)
// (:78-102): a spring of rest x = s.r + i.r (weakly cast to float32 in dx = current - x) and stiffness k/2
// (float32 in f_size = -dx*k), applied to s and then to i.  The term a pair adds to either end does not
// depend on which end is s (norm and r_s + r_i are symmetric), so mass q receives, in the reference's order:
// every partner j < q (outer loop at j), then every partner j != q ascending (outer loop at q), then every
// partner j > q (outer loop at j).  rs = this lane's Point.r (the env pass overwrites it with 3 / 1).
// With a bounce_set (Point.bounce(k, other=<list>) on a subset of callers): bs = this lane's bits (1 calls, 2 in the
// list); q receives, in the same three phases, the terms of callers j < q when q is listed, its own call's terms
// against the listed j != q when q calls, then the terms of callers j > q when q is listed (bs = 3: every point).
__device__ __forceinline__ void pair_bounce(float kh, double rs, int bs, const float *p3, float mf, int lane, int M,
                                            bool is_mass, float &ax, float &ay, float &az) {
    const int gb = lane & ~(M - 1), q = lane & (M - 1);
    const double md = (double)mf, ym = 1.0 / md;
    for (int ph = 0; ph < 3; ph++) {
        for (int pj = 0; pj < M; pj++) {
            const int src = (gb + pj) << 2;
            const float ox = lane_gather(p3[0], src), oy = lane_gather(p3[1], src), oz = lane_gather(p3[2], src);
            const double orad = lane_gather_d(rs, src);
            const int obs = __builtin_amdgcn_ds_bpermute(src, bs);
            const bool on = ph == 1 ? pj != q && (bs & 1) && (obs & 2)
                                    : (ph == 0 ? pj < q : pj > q) && (obs & 1) && (bs & 2);
            if (!is_mass || !on) continue;
            const float d0 = ox - p3[0], d1 = oy - p3[1], d2 = oz - p3[2];   // partner - self
            const float cur = np_norm3(d0, d1, d2);
            const double x = rs + orad;
            if (!((double)cur <= x)) continue;
            const float dx = cur - (float)x;                                  // engine.py:96
            const float nf = -((-dx) * kh);                                   // -f_size, :75,100
            bounce_term(cur, nf, d0, d1, d2, md, ym, ax, ay, az);
        }
    }
}

// pair_mode bit 8: G2 Point.gravity (gravity_vec, g2_gravity_term) over the walker's M lanes: every a zeroed first
// (gym/optimized_engine.py:174-175; the walker has M >= 4 masses here), partners in ascending order by ds_bpermute.
__device__ __forceinline__ void pair_g2_gravity(double g, const float *p3, float mf, int lane, int M, bool is_mass,
                                                float &ax, float &ay, float &az) {
    const int gb = lane & ~(M - 1), q = lane & (M - 1);
    const double md = (double)mf, ym = 1.0 / md;
    ax = 0.f; ay = 0.f; az = 0.f;
    for (int pj = 0; pj < M; pj++) {
        const int src = (gb + pj) << 2;
        const float ox = lane_gather(p3[0], src), oy = lane_gather(p3[1], src), oz = lane_gather(p3[2], src);
        const float om = lane_gather(mf, src);
        if (!is_mass || pj == q) continue;
        const double mo = (double)om;
        g2_gravity_term(((-g) * (pj < q ? mo : md)) * (pj < q ? md : mo), ox - p3[0], oy - p3[1], oz - p3[2], mf, ym,
                        ax, ay, az);
    }
}

// The pair passes of one wave (pair_mode != 0): gravity, coulomb, bounce, each over every walker of the wave.
// Per-mass charges / radii are loaded here, not in lean_load, so the default path carries no extra registers.
__device__ __forceinline__ void pair_forces(const wg_batch &b, const KParams &kp, const float *p3, float mf,
                                         uint32_t pl, int lane, int M, bool is_mass, float &ax, float &ay,
                                         float &az) {
    if (kp.pair_mode & 1) pair_central(kp.pair_g, (double)mf, p3, mf, lane, M, is_mass, ax, ay, az);
    if (kp.pair_mode & 2) {
        const double e = (b.charge && is_mass) ? b.charge[pl] : kp.pair_e;
        pair_central(kp.pair_k, e, p3, mf, lane, M, is_mass, ax, ay, az);
    }
    if (kp.pair_mode & 4) {
        const double rs = is_mass ? b.radius[pl] : 0.0;
        const int bs = b.bounce_set ? (is_mass ? (int)b.bounce_set[pl] : 0) : 3;
        pair_bounce(kp.bounce_kh, rs, bs, p3, mf, lane, M, is_mass, ax, ay, az);
    }
    if (kp.pair_mode & 8) pair_g2_gravity(kp.pair_g, p3, mf, lane, M, is_mass, ax, ay, az);
    if (kp.pair_mode & 16) {
        const double e = (b.charge && is_mass) ? b.charge[pl] : kp.pair_e;
        pair_central(kp.pair_k, e, p3, mf, lane, M, is_mass, ax, ay, az, true);
    }
}

// Spring terms of the lean kernels, interleaved per edge.  (Three f64 and three f32 planes make the edge lanes'
// stores conflict-free, but the mass loop's random reads then take three separate 8-B reads per term instead of
// one ds_read2_b64 + one ds_read_b64: 48.1 against 47.3 us per launch, profiles/r02_ab_soa_canonical.json.)


typedef TermsAoS LeanTerms;
__device__ __forceinline__ LeanTerms lean_terms(char *sl, const LeanGeo &lg) {
    return TermsAoS{reinterpret_cast<double *>(sl), reinterpret_cast<float *>(sl + lg.off_df)};
}

// One wave's tile after its loads: the edge lanes leave the spring term t and the damping force df of every
// edge in LDS, then each mass lane walks its incidence list, dividing by m as the reference does (mass_step).
// RES (walker_rollout_lean): the tile's state stays in L across steps; it is written to HBM only when `last`.
template <bool IN3D, int NE, bool RES = false>
__device__ __forceinline__ void lean_compute(const wg_batch &b, const KParams &kp, const KOut &o,
                                             const LeanGeo &lg, char *sl, const LeanTile &t, int lane,
                                             LeanIn<NE> &L, bool last = true) {
    const bool store = !RES || last;
    const int M = b.M, K = b.K, A = b.A;
    const int w0 = t.w0, nE = t.nE;
    const int wl = t.wl, q = t.q, mu_wl = t.mu_wl, mu_ua = t.mu_ua;
    const bool is_mass = t.is_mass, is_mus = t.is_mus, acts = t.acts;
    const uint32_t pl = t.P0 + lane, ul = t.U0 + lane;   // this lane's mass / muscle
    // slice: spring terms t (f64 x3) | df (f32 x3) | incidence words | muscle x
    const LeanTerms ts = lean_terms(sl, lg);
#ifdef WG_STAMPS
    const int stamp_wave = t.w0 / lg.wpw;   // (the tile index, as the kernel's own stamps use)
#endif
    uint32_t *s_inc = reinterpret_cast<uint32_t *>(sl + lg.off_inc);
    float *s_x = reinterpret_cast<float *>(sl + lg.off_x);
    const float mf = L.mf;
    const bool pin = L.pin != 0;
    // (NE = 1: glibc's powf tables in registers, lane l < 32 holding entry l of each)
    double sq_tl = 0.0, sq_te = 0.0;
    if (NE == 1 && !RES) {   // (not the resident kernel: its carried state holds the registers)
        sq_tl = PW_LOG2_TAB[lane & 31];
        sq_te = pw_asdouble(PW_EXP2_TAB[lane & 31]);
    }

    // ================= act (gym/optimized_walker.py:27-43,164-172); the incidence lists go to LDS first
    if (!RES) {   // (the resident kernel writes them once, before its first step)
#pragma unroll
        for (int it = 0; it < NE; it++)
            if (lane + 64 * it < nE) s_inc[lane + 64 * it] = L.gi[it];
        if (lane == 0) s_inc[nE] = 0u;   // the read-ahead pad after the last list (mass_accumulate_v2)
    }
    float x = L.x;
    if (acts) {
        x = (kp.action_mode == 1) ? ((L.a != 0.f) ? x + L.stp : x - L.stp) : x + L.a;
        if (L.lo > x) x = L.lo;     // Python max(x, originx*minl)
        if (L.hi < x) x = L.hi;     // Python min(x, originx*maxl)
        if (store) *WG_ST(b.muscle_x, ul, 1) = x;
    }
    if (is_mus) s_x[lane] = x;
    double ym = recip_m(mf);        // RN64(1/m) of this lane's mass: every /m below is exact from it
    // (opaque: otherwise the compiler turns (float)ym, which is RN32(1/m), into a second, float32 IEEE division)
    if (!RES) asm volatile("" : "+v"(ym));
    wave_sync();
    STAMP(2);

    // ================= diverged walkers (round 6): every mass of the walker has a NaN position component, is not pinned
    // and has a spring.  Then every spring term of the walker is NaN (norm, dx, f and the direction all are: Python's
    // max(NaN, r) keeps NaN, gym/engine.py:73-75), so each mass's a, and after run1 its v and pos, are NaN in all three
    // components; its contact test (pos_y - ground < 0) is false; the muscle lengths still follow the actions.  The
    // walker's lanes step benign finite stand-ins (mass q at (q, 0, 0), at rest) so that no exact cold path runs for it,
    // and its state, outputs and sums are then set to what the reference computes: NaN (NaN payloads aside).  A
    // walker only partly NaN, or with an inf, steps exactly as before.  Pair passes keep the plain path.
    bool dead = false;
    if ((!RES || NE == 1) && kp.pair_mode == 0) {   // (the resident kernel: its latency-bound NE = 1 instance)
        // (the common test reads the positions only, the first loads to land: the pin / incidence words are waited for
        // only in the rare branch, so the springs do not start later)
        const bool nanp = is_mass && (__builtin_isnan(L.p3[0]) || __builtin_isnan(L.p3[1]) || __builtin_isnan(L.p3[2]));
        if (__builtin_expect(__ballot(nanp) != 0ull, 0)) {   // wave-uniform, rare
            const unsigned long long db = __ballot(nanp && !pin && L.io1 > L.io0);
            const unsigned long long gm = (M == 64) ? ~0ull : (((1ull << M) - 1ull) << (lane & ~(M - 1)));
            dead = is_mass && (db & gm) == gm;
            if (dead) {
                L.p3[0] = (float)q; L.p3[1] = 0.f; L.p3[2] = 0.f;
                L.v3[0] = 0.f; L.v3[1] = 0.f; L.v3[2] = 0.f;
            }
        }
    }

    // ================= springs: gym/engine.py:78-102 + gym/optimized_walker.py:92-106 =================
    bool gtiny = false;   // a damping force of this lane's springs outside the mass loop's exact quotient range
    const bool pos_ok = __all(fexp3(L.p3[0], L.p3[1], L.p3[2]) >= -55);   // (spring_terms)
    // endpoint state from the mass lanes by ds_bpermute: every lane takes part (inactive sources read as 0).
    // (Issuing pass it + 1's gathers before pass it's arithmetic needs 90 VGPRs, 5 waves per SIMD: 48.5 against
    // 47.8 us per launch, profiles/r02_ab_spring_pipe.json.)
    struct Gath { float v[12]; };
    auto gather = [&](int it, Gath &g) {
        const int le = lane + 64 * it;
        const int ewl = fdiv(le, K, lg.invK);
        const uint32_t ij = L.er[it].ij;
        // (M | 64 is a power of two: the walker's first lane is a shift; 24-bit products below, one VALU each)
        const int bi = ((ewl << lg.lgM) + edge_i(ij)) << 2, bj = ((ewl << lg.lgM) + edge_j(ij)) << 2;
#pragma unroll
        for (int c = 0; c < 3; c++) {
            if (WG_ABLATE & 512) {   // (ablation: no gathers, the lane's own state at both ends, shifted)
                g.v[c] = L.p3[c]; g.v[3 + c] = L.p3[c] + (float)(bj - bi); g.v[6 + c] = L.v3[c]; g.v[9 + c] = L.v3[c];
                continue;
            }
            g.v[c] = lane_gather(L.p3[c], bi); g.v[3 + c] = lane_gather(L.p3[c], bj);
            g.v[6 + c] = lane_gather(L.v3[c], bi); g.v[9 + c] = lane_gather(L.v3[c], bj);
        }
    };
    auto spring = [&](int it, const Gath &g) {
        const int le = lane + 64 * it;
        const EdgeRec e = L.er[it];
        const int ewl = fdiv(le, K, lg.invK), ew = le - (int)__umul24(ewl, K);
        // the muscle's rest length read unconditionally (clamped index), then selected by value: a select
        // between the LDS slot and e.rest became a pointer select (flat load from a stack copy of e)
        const bool mus = le < nE && ew < A;
        const float xs = s_x[mus ? (int)__umul24(ewl, A) + ew : 0];
        const float xr = mus ? xs : e.rest;
        if (le < nE) {
            if (WG_ABLATE & 1) {   // profiling builds only: no spring arithmetic
                ts.put(le, xr + g.v[0] + g.v[3] + g.v[6] + g.v[9], g.v[1] + g.v[4] + g.v[7] + g.v[10],
                       g.v[2] + g.v[5] + g.v[8] + g.v[11], e.k, e.c, 0.f);
            } else {
                spring_edge_regs(e, le, xr, g.v[0], g.v[1], g.v[2], g.v[3], g.v[4], g.v[5], g.v[6], g.v[7], g.v[8],
                                 g.v[9], g.v[10], g.v[11], ts, 0, gtiny, pos_ok);   // lean path: spring_mode 0 only
            }
        }
    };
#pragma unroll
    for (int it = 0; it < NE; it++) {
        // no early loop exit: it keeps er[] in registers (a reference under a `break` made hipcc park the rest
        // lengths in scratch right after their loads, serialising them)
        if (64 * it >= nE) continue;                       // wave-uniform
        if ((WG_ABLATE & 4096) && it == NE - 1 && it > 0) {   // (ablation: the last spring pass's terms as zeros)
            const int le = lane + 64 * it;
            if (le < nE) ts.put(le, 0.0, 0.0, 0.0, 0.f, 0.f, 0.f);
            continue;
        }
        Gath g;
        gather(it, g);
        spring(it, g);
    }
    wave_sync();
    // any spring of the wave with a damping force outside the exact range: every mass loop of the wave divides by m with
    // IEEE divisions (rare: damping forces below 2^-80)
    const bool wave_tiny = __any(gtiny);
    STAMP(3);

    // ================= masses: ordered accumulation, env forces, Point.run1 =================
    // the env forces' quotients (m, v and y of the step's start only) ahead of the mass loop, once the spring records'
    // registers are free: after the loop only their ordered additions remain (the resident kernel, whose state
    // registers are tight, keeps them in mass_tail)
    EnvTerms et{};
    if (!RES) et = env_terms(kp, mf, (float)ym, L.v3[0], L.v3[1], L.v3[2]);
    float px = 0.f, py = 0.f, pz = 0.f, vx = 0.f, vy = 0.f, vz = 0.f, ax = 0.f, ay = 0.f, az = 0.f;
    float nv = 0.f, ke = 0.f, pe = 0.f;
    bool hit = false;
    if (is_mass) {
        const int r1 = (WG_ABLATE & 2) ? min(L.io1, L.io0 + 1) : L.io1;
        const int lb = wl * K;
        // (the resident kernel keeps the XOR sign form: 5 fewer registers where its carried state is live)
        if (!RES)
            mass_accumulate_v2(ts, reinterpret_cast<const uint16_t *>(s_inc) + 2 * lb, lb, L.io0, r1, mf, ym, ax, ay, az,
                               wave_tiny);
        else
            mass_accumulate<LeanTerms, !RES>(ts, reinterpret_cast<const uint16_t *>(s_inc) + 2 * lb, lb, L.io0, r1, mf,
                                             ax, ay, az, 0, wave_tiny);
    }
    // every lane (gathers); the resident kernel runs pair-free batches only (wg_rollout falls back to wg_step)
    if (!RES && kp.pair_mode) pair_forces(b, kp, L.p3, mf, pl, lane, M, is_mass, ax, ay, az);
    if (is_mass) {
        mass_tail(kp, mf, (float)ym, L.p3, L.v3, px, py, pz, vx, vy, vz, ax, ay, az, hit, pin,
                  !RES ? &et : nullptr);
        if (dead) {   // (a diverged walker, above: what the reference computes)
            px = __builtin_nanf(""); py = px; pz = px; vx = px; vy = px; vz = px; ax = px; ay = px; az = px;
            hit = false;
        }
        if (b.radius && store) b.radius[pl] = hit ? 3.0 : 1.0;   // p.r = 3 / p.r = 1 (gym/optimized_env.py:156,175)
        nv = np_norm3(vx, vy, vz);
        if (!(NE == 1 && !RES)) ke = dead ? nv : mf * np_sq<NE == 1>(nv);   // p.m * norm(p.v) ** 2 (optimized_env.py:242)
        pe = (float)((double)mf * kp.g) * (py - kp.ground);
    }
    if (NE == 1 && !RES) {   // every lane (table gathers); lanes past the masses square 0
        const float sq = np_sq_wave(dead ? 0.f : nv, sq_tl, sq_te);
        if (is_mass) ke = dead ? nv : mf * sq;
    }
    STAMP(4);

    // ================= per-walker reductions (wave shuffles) + outputs (gym/optimized_env.py:189-248)
    const int gbase = lane & ~(M - 1);
    const WalkerSums ws = (WG_ABLATE & 4) ? WalkerSums{px, py, pz, py, nv, ke, pe}   // (ablation: no reductions)
                                          : walker_sums(px, py, pz, nv, ke, pe, gbase, M, lane);
    const float sx = ws.sx, sy = ws.sy, sz = ws.sz, ysum = ws.ysum, vsum = ws.vsum, ksum = ws.ksum, psum = ws.psum;
    const unsigned long long gmask = (M == 64) ? ~0ull : (((1ull << M) - 1ull) << gbase);
    const unsigned long long hb = __ballot(is_mass && (py - kp.ground < 0.f));   // contacts after run1 (:200)
    const unsigned long long sb = __ballot(is_mass && nv < 0.1f);
    // M | 64 is a power of two: x / M == x * (1/M) exactly (the same real number, rounded once)
    const float midx = sx * lg.invM, midy = sy * lg.invM, midz = sz * lg.invM;
    if (is_mass) {
        if (store) {
            float *gpo = WG_ST(b.pos, pl, 3), *gvo = WG_ST(b.vel, pl, 3), *gao = WG_ST(b.acc, pl, 3);
            gpo[0] = px; gpo[1] = py; gpo[2] = pz;
            gvo[0] = vx; gvo[1] = vy; gvo[2] = vz;
            gao[0] = ax; gao[1] = ay; gao[2] = az;
            if (b.contact) at_u32w(b.contact, pl) = (uint8_t)hit;
        }
        if (q == 0) {
            const uint32_t wg = (uint32_t)(w0 + wl);
            const int steps = L.wsteps + 1;
            if (store) *WG_ST(b.steps, wg, 1) = steps;
            if (RES) L.wsteps = steps;
            if (o.steps) *WG_ST(o.steps, wg, 1) = steps;
            const float cy = ysum * lg.invM;
            if (o.reward) {
                const float vpen = (-(vsum * lg.invM)) * 0.1f;
                *WG_ST(o.reward, wg, 1) = (cy + vpen) + neg_half_count((int)__popcll(hb & gmask));
            }
            if (o.done) {
                int done = steps >= kp.max_steps;
                if (!done && cy < kp.done_y) done = 1;
                if (!done && steps > 100) done = (sb & gmask) == gmask;
                at_u32w(o.done, wg) = (uint8_t)done;
            }
            if (o.centroid) {
                float *c = WG_ST(o.centroid, wg, 3);
                c[0] = midx; c[1] = midy; c[2] = midz;
            }
            if (o.energy) *WG_ST(o.energy, wg, 1) = 0.5f * ksum + psum;
        }
    }

    STAMP(5);
    // ================= observation rows: Creature.getstat (gym/optimized_walker.py:129-162) =========
    if (o.obs && !(WG_ABLATE & 16)) {
        // straight from registers: lane q's 3d values are one contiguous piece of its walker's row, stored as d-float
        // vectors; the wave's pieces tile the rows, and the L2 merges them into whole lines
        constexpr int d = IN3D ? 3 : 2, per = 3 * d;
        const int stride = o.obs_stride, nmid = kp.conmid ? 3 : 0;
        typedef float fvd __attribute__((ext_vector_type(d), aligned(4)));
        if (is_mass) {
            const uint32_t row0 = (uint32_t)(w0 + wl) * (uint32_t)stride;   // the row's first element
            // G1 getstat (midform 2, gym/walker.py:88-96) subtracts the SUM of positions
            const float mm[3] = {kp.midform == 2 ? sx : midx, kp.midform == 2 ? sy : midy, kp.midform == 2 ? sz : midz};
            const float pm[3] = {px, py, pz}, vm[3] = {vx, vy, vz}, am[3] = {ax, ay, az};
            fvd vp, vv, va;
#pragma unroll
            for (int c = 0; c < d; c++) {
                vp[c] = kp.midform ? (pm[c] - mm[c]) * kp.pk : pm[c] * kp.pk;
                vv[c] = vm[c] * kp.vk;
                va[c] = am[c] * kp.ak;
            }
            float *dst = WG_ST(o.obs, row0 + per * q, 1);   // (a 3-vector's type is 16 B: no array indexing over fvd)
            *reinterpret_cast<fvd *>(dst) = vp;
            *reinterpret_cast<fvd *>(dst + d) = vv;
            *reinterpret_cast<fvd *>(dst + 2 * d) = va;
            if (q == 0) {
                if (nmid) {
                    float *mrow = WG_ST(o.obs, row0 + per * M, 1);
                    mrow[0] = kp.midform ? mm[0] : 0.f; mrow[1] = kp.midform ? mm[1] : 0.f;
                    mrow[2] = kp.midform ? mm[2] : 0.f;
                }
                for (int r = per * M + nmid + A; r < stride; r++) *WG_ST(o.obs, row0 + r, 1) = 0.f;
            }
        }
        if (is_mus) *WG_ST(o.obs, (uint32_t)(w0 + mu_wl) * (uint32_t)stride + per * M + nmid + mu_ua, 1) = x * kp.mk;
    }
    if (RES) {   // the next step starts from this one's state (Point.pos/v, Muscle.x), in registers
        L.p3[0] = px; L.p3[1] = py; L.p3[2] = pz;
        L.v3[0] = vx; L.v3[1] = vy; L.v3[2] = vz;
        L.x = x;
    }
    STAMP(6);
#ifdef WG_STAMPS
    if (lane == 0 && stamp_wave < (1 << 16)) {   // slot 7: HW_ID (gfx9 hwreg 4) | XCC_ID (gfx940+ hwreg 20) << 32
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        g_stamps[stamp_wave * 8 + 7] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
    }
#endif
}

// NE spring passes per wave need up to 8 x 16-B records in registers: 6 waves per SIMD hold up to NE 4 without
// spills, NE 8 (up to 512 springs per 64 lanes) gets the 4-wave register budget.
constexpr int lean_waves(int NE) { return NE >= 8 ? 4 : 6; }

// One tile (64 / M walkers) per wave; waves never wait for one another.
template <bool IN3D, int NE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(lean_waves(NE)))) void walker_step_lean(
    wg_batch b, KParams kp, const float *__restrict__ action, int action_cols, int action_stride, KOut o,
    LeanGeo lg) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // the wave index as a wave-uniform (scalar) value: the tile's walker range and element bases are then SALU
    // products, not per-lane v_mul_lo_u32
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int blk = (kp.xcd & 2) ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int tile = blk * lg.wpb + wv;
    if (tile * lg.wpw >= b.N) return;
#ifdef WG_STAMPS
    const int stamp_wave = tile;
#endif
    STAMP(0);
    const LeanTile t = lean_tile_of(b, action, action_cols, lg, tile, lane);
    LeanIn<NE> L;
    // load-phase wave priority: this wave's HBM requests leave before other waves' arithmetic
    if (kp.prio) __builtin_amdgcn_s_setprio(2);
    lean_load<NE>(b, kp, action, action_stride, t, lane, L);
    if (kp.prio) __builtin_amdgcn_s_setprio(0);
    STAMP(1);
    lean_compute<IN3D, NE>(b, kp, o, lg, smem + wv * lg.slice, t, lane, L);
}

// NE = 1, the latency-bound small batches (Balance-4096: 512 waves, one per SIMD, the launch as long as its slowest
// wave's dependent chain): the lean step with its leading arguments PRELOADED into SGPRs by the dispatch (build.py:
// -mllvm -amdgpu-kernarg-preload-count=10; the option preloads leading pointer / scalar arguments only, <= 14 SGPRs).
// These ten are everything the tile index and the first vector loads (pos, vel, spring records, incidence words) need,
// so those loads issue at the wave's first instructions while one scalar round fetches the rest; nblkx = the workgroup
// count | the XCD-order flag << 30 | the load-phase priority flag << 31.  Left to the compiler, walker_step_lean's
// by-value structs had cost three dependent scalar rounds before the first vector load.  Balance-4096, one launch per
// step, same box, interleaved: round 5's prologue 5.33 us, the same arguments in one scalar round 5.01
// (profiles/r06b_ab_balance4096_prologue.json), preloaded 2.5 % below that (profiles/r06e_ab_*).
template <bool IN3D>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(lean_waves(1)))) void walker_step_lean1(
    float *pos, float *vel, const wg_edge *edges, const uint16_t *inc, int N, int M, int K, int wpw, int wpb, int nblkx,
    wg_batch b, KParams kp, const float *__restrict__ action, int action_cols, int action_stride, KOut o, LeanGeo lg) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    b.pos = pos; b.vel = vel; b.edges = edges; b.inc = inc; b.N = N; b.M = M; b.K = K;
    lg.nblk = nblkx & 0x3fffffff; lg.wpw = wpw; lg.wpb = wpb;
    kp.prio = (int)((unsigned)nblkx >> 31);
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bid = blockIdx.x, xb = xcd_block(bid, lg.nblk);
    const int blk = (nblkx & 0x40000000) ? xb : bid;
    const int tile = blk * lg.wpb + wv;
    if (tile * lg.wpw >= b.N) return;
#ifdef WG_STAMPS
    const int stamp_wave = tile;
#endif
    STAMP(0);
    const LeanTile t = lean_tile_of(b, action, action_cols, lg, tile, lane);
    LeanIn<1> L;
    if (kp.prio) __builtin_amdgcn_s_setprio(2);
    lean_load<1>(b, kp, action, action_stride, t, lane, L);
    if (kp.prio) __builtin_amdgcn_s_setprio(0);
    STAMP(1);
    lean_compute<IN3D, 1>(b, kp, o, lg, smem + wv * lg.slice, t, lane, L);
}

// n_steps env steps in one launch (wg_rollout): the tile's static inputs (spring records, incidence lists, masses,
// muscle bounds) are loaded once and its state (pos, vel, muscle x, step counter) stays in registers from step to
// step; each step reads its actions (the next step's are in flight while this one computes) and writes its
// outputs; pos / vel / acc / contact / muscle x / steps go to HBM after the last step.  Same arithmetic as
// walker_step_lean, step for step (bit-identical to n_steps single-step launches).
template <bool IN3D, int NE>
// (register budget: 5 waves per SIMD since the scalar wave index, 16 B of scratch at NE 3-4: 35.49 against 36.07 us per
// step at 4, profiles/r04l_ab_resident.json)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NE >= 8 ? 4 : 5))) void walker_rollout_lean(
    wg_batch b, KParams kp, const float *__restrict__ action, int action_cols, int action_stride, int64_t action_step,
    KOut o, int n_steps, LeanGeo lg) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tile = blockIdx.x * lg.wpb + wv;
    if (tile * lg.wpw >= b.N) return;
#ifdef WG_STAMPS
    const int stamp_wave = tile;
#endif
    const LeanTile t = lean_tile_of(b, action, action_cols, lg, tile, lane);
    LeanIn<NE> L;
    if (kp.prio) __builtin_amdgcn_s_setprio(2);
    lean_load<NE>(b, kp, action, action_stride, t, lane, L);
    if (kp.prio) __builtin_amdgcn_s_setprio(0);
    {   // the incidence lists are static: into LDS once
        uint32_t *s_inc = reinterpret_cast<uint32_t *>(smem + wv * lg.slice + lg.off_inc);
#pragma unroll
        for (int it = 0; it < NE; it++)
            if (lane + 64 * it < t.nE) s_inc[lane + 64 * it] = L.gi[it];
    }
#pragma clang loop unroll(disable)
    for (int s = 0; s < n_steps; s++) {
        // the lane index made opaque each step: its derived addresses and masks are recomputed in the step (a few
        // VALU) instead of being hoisted out of the loop and held in registers (spilled) across all of it
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const LeanTile ts = lean_tile_of(b, action, action_cols, lg, tile, ln);
        float a_next = 0.f;                        // the next step's action, in flight while this step computes
        if (ts.acts && s + 1 < n_steps)
            a_next = action[(size_t)(s + 1) * (size_t)action_step +
                            (size_t)(uint32_t)(ts.w0 + ts.mu_wl) * (uint32_t)action_stride + (uint32_t)ts.mu_ua];
        KOut os = o;
        if (os.obs) os.obs += (size_t)s * os.obs_step;
        if (os.reward) os.reward += (size_t)s * os.out_step;
        if (os.done) os.done += (size_t)s * os.out_step;
        if (os.energy) os.energy += (size_t)s * os.out_step;
        if (os.centroid) os.centroid += 3 * (size_t)s * os.out_step;
        if (os.steps) os.steps += (size_t)s * os.out_step;
        // the same for the static inputs (the mass's 1/m, the springs' endpoint indices are re-derived per step)
        asm volatile("" : "+v"(L.mf), "+v"(L.io0), "+v"(L.io1), "+v"(L.lo), "+v"(L.hi), "+v"(L.stp));
#pragma unroll
        for (int it = 0; it < NE; it++) asm volatile("" : "+v"(L.er[it].ij), "+v"(L.er[it].rest), "+v"(L.er[it].k),
                                                     "+v"(L.er[it].c));
        lean_compute<IN3D, NE, true>(b, kp, os, lg, smem + wv * lg.slice, ts, ln, L, s == n_steps - 1);
        L.a = a_next;
        wave_sync();   // this step's LDS reads stay ahead of the next step's writes
    }
}

// ------------------------------------------------------------------ ragged wave kernel
// Mixed-topology batches whose walkers all have M_w <= 64 (wg_batch.ragged = 2).  The host sorts the walkers by
// size and packs them into wave tiles (wg_plan_waves): contiguous stored walkers with at most 64 masses, 64
// muscles, RW_MAXW walkers and 64 * NE springs in all.  One wave per tile and no workgroup barrier, with the lean
// kernel's arithmetic: one mass per lane (the tile's walkers side by side), the springs in NE passes of 64 lanes
// with the endpoints' state gathered by ds_bpermute, each mass lane walking its incidence list in reference
// order.  What differs from the uniform lean kernel is bookkeeping: a lane finds its walker by counting the walker
// starts at or below it (v_readlane of the walker lanes' offsets); per-walker reductions run 8 lanes per walker over an LDS copy of the
// per-mass terms in numpy's orders (as walker_step_kernel); observation rows are assembled in LDS and streamed to
// the caller's rows (wg_batch.row), zero padded to the stride.
constexpr int RW_MAXW = 32;   // walkers per wave tile (planner cap)
__device__ int g_plan_error;  // set (vector atomic) by a wave-kernel tile beyond the caps; read by wg_plan_errors

struct RagGeo {
    int wpb;                  // waves per workgroup
    int slice;                // LDS bytes per wave
    int off_df, off_inc, off_x, off_wo;   // byte offsets in the slice (spring terms at 0)
};


template <bool IN3D, int NE>
// LDS: ~5.8 KB per wave at NE 2 (27 waves per CU); NE 4 / 8 tiles need more LDS and registers
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NE >= 8 ? 4 : NE >= 4 ? 5 : 6))) void walker_step_waves(
    wg_batch b, KParams kp, const float *__restrict__ action, int action_cols, int action_stride, KOut o,
    const int32_t *__restrict__ plan, int ntiles, RagGeo rg) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    // the wave index as a wave-uniform (scalar) value: the plan entries and the tile's bases are then scalar loads
    // (scalar cache, lgkmcnt) rather than vector loads each waited for before the next one can be addressed
    const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int blk = (kp.xcd & 1) ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int tile = blk * rg.wpb + wv;
    if (tile >= ntiles) return;
#ifdef WG_STAMPS
    const int stamp_wave = tile;
#endif
    STAMP(0);
    char *sl = smem + wv * rg.slice;
    const TermsAoS ts{reinterpret_cast<double *>(sl), reinterpret_cast<float *>(sl + rg.off_df)};
    uint32_t *s_inc = reinterpret_cast<uint32_t *>(sl + rg.off_inc);
    float *s_x = reinterpret_cast<float *>(sl + rg.off_x);
    int *s_mo = reinterpret_cast<int *>(sl + rg.off_wo);              // [RW_MAXW + 1] tile-local offsets
    int *s_eo = s_mo + (RW_MAXW + 1), *s_uo = s_eo + (RW_MAXW + 1), *s_row = s_uo + (RW_MAXW + 1);
    float *s_mid = reinterpret_cast<float *>(s_row + RW_MAXW);          // [RW_MAXW * 3] each walker's mean position
    // after the mass loop: per-mass terms in the spring-term region, pos [64*3] | |v| | m|v|^2 | m g (y-ground),
    // then the obs staging; the walker partials [RW_MAXW * 8] in the damping region
    float *s_tp = reinterpret_cast<float *>(sl);
    float *s_tn = s_tp + 192, *s_tk = s_tn + 64, *s_te = s_tk + 64;
    float *s_red = reinterpret_cast<float *>(sl + rg.off_df);

    // ================= loads: the tile's walker offsets first (the lane maps need them), then everything else
    if (kp.prio) __builtin_amdgcn_s_setprio(2);
    const int w0 = plan[tile], w1 = plan[tile + 1], nw = w1 - w0;
    const int P0 = b.mass_off[w0], E0 = b.edge_off[w0], U0 = b.muscle_off[w0];
    const int nP = b.mass_off[w1] - P0, nE = b.edge_off[w1] - E0, nU = b.muscle_off[w1] - U0;
    // a plan tile beyond the wave's caps (a caller-made plan, ADVICE r2: wg_step trusts device plans) would write past
    // this wave's LDS slice: such a tile is skipped — its walkers keep their state — and the launch reports it through
    // g_plan_error (wg_plan_errors); wg_plan_waves never produces one
    if (nw < 1 || nw > RW_MAXW || nP < 1 || nP > 64 || nU > 64 || nE > 64 * NE) {
        if (lane == 0) atomicOr(&g_plan_error, 1);
        return;
    }
    // every vector load that needs only the tile's bases, issued back to back from clamped (valid) indices: a load
    // under a per-lane branch whose result the register allocator copies waits right there, and with vmcnt counting
    // in order that wait covers every load before it.  Lanes past the tile's walkers / masses / springs / muscles
    // load a duplicate and are given the reference values (zeros) once everything has landed.
    const bool is_mass = lane < nP, is_mus = lane < nU;
    const int lw = min(lane, nw), lr = min(lane, nw - 1);
    // (addresses as SGPR base + 32-bit byte offset: the saddr form of global_load, no 64-bit VALU arithmetic)
    int wmo = at_u32(b.mass_off, 4u * (w0 + lw)) - P0, weo = at_u32(b.edge_off, 4u * (w0 + lw)) - E0;
    int wuo = at_u32(b.muscle_off, 4u * (w0 + lw)) - U0;
    int wsteps = at_u32(b.steps, 4u * (w0 + lr));
    const int lp = P0 + min(lane, max(nP, 1) - 1);   // a tile has at least one mass
    float p3[3], v3[3];
    {
        const float *gp = &at_u32(b.pos, 12u * lp), *gv = &at_u32(b.vel, 12u * lp);
        p3[0] = gp[0]; p3[1] = gp[1]; p3[2] = gp[2];
        v3[0] = gv[0]; v3[1] = gv[1]; v3[2] = gv[2];
    }
    float mf = at_u32(b.mass, 4u * lp);
    EdgeRec er[NE];
    uint32_t gi[NE];
    if (nE > 0) {
#pragma unroll
        for (int it = 0; it < NE; it++) {
            const uint32_t le = E0 + min(lane + 64 * it, nE - 1);
            const uint4 v = at_u32(reinterpret_cast<const uint4 *>(b.edges), 16u * le);
            er[it] = EdgeRec{v.x, __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w)};
            gi[it] = at_u32(reinterpret_cast<const uint32_t *>(b.inc), 4u * le);
        }
    }
    float mx = 0.f, mlo = 0.f, mhi = 0.f, mst = 0.f;
    if (nU > 0) {
        const uint32_t lu = U0 + min(lane, nU - 1);
        mx = at_u32(b.muscle_x, 4u * lu);
        if (action) {
            const float2 bd = at_u32(reinterpret_cast<const float2 *>(b.muscle_bounds), 8u * lu);
            mlo = bd.x; mhi = bd.y;
            if (kp.action_mode == 1) mst = at_u32(b.muscle_stride, 4u * lu);
        }
    }
    int wrow = w0 + lr, pin = 0;
    if (b.row && !(WG_ABLATE & 2048)) wrow = at_u32(b.row, 4u * (w0 + lr));   // (ablation 2048: rows in stored order)
    if (b.pinned) pin = at_u32(b.pinned, (uint32_t)lp);
    // lane -> walker maps (tile-local offsets in LDS)
    if (lane <= nw) { s_mo[lane] = wmo; s_eo[lane] = weo; s_uo[lane] = wuo; }
    if (lane < nw) s_row[lane] = wrow;
    // lane -> walker maps by counting the walker starts at or below the lane: the starts are in the walker lanes'
    // registers (v_readlane, no LDS round trips; a tile has few walkers); NE spring passes map their edge slots too
    int mw = 0, uw = 0, eww[NE];
#pragma unroll
    for (int it = 0; it < NE; it++) eww[it] = 0;
    for (int w = 1; w < nw; w++) {
        const int so = __builtin_amdgcn_readlane(wmo, w), se = __builtin_amdgcn_readlane(weo, w);
        const int su = __builtin_amdgcn_readlane(wuo, w);
        mw += lane >= so;
        uw += lane >= su;
#pragma unroll
        for (int it = 0; it < NE; it++) eww[it] += lane + 64 * it >= se;
    }
    if (!is_mass) mw = 0;
    if (!is_mus) uw = 0;
    wave_sync();
    const int mlm = s_mo[mw], mlb = s_eo[mw];
    // inc_off (M_w + 1 entries per walker) and the action: the second (and last) round of vector loads
    const uint32_t io = (uint32_t)lp + (uint32_t)(w0 + mw);
    int io0 = at_u32(b.inc_off, 2u * io), io1 = at_u32(b.inc_off, 2u * io + 2u);
    const int ua = lane - s_uo[uw];                                      // this lane's muscle in walker uw
    const bool acts = action != nullptr && is_mus && ua < action_cols;
    float act = 0.f;
    if (action && action_cols > 0)
        act = at_u32(action, 4u * ((uint32_t)s_row[uw] * (uint32_t)action_stride + (uint32_t)min(max(ua, 0), action_cols - 1)));
    // the reference values of the lanes past the tile's masses / muscles (the loads above read duplicates)
    if (!is_mass) {
        p3[0] = 0.f; p3[1] = 0.f; p3[2] = 0.f; v3[0] = 0.f; v3[1] = 0.f; v3[2] = 0.f;
        mf = 0.f; pin = 0; io0 = 0; io1 = 0;
    }
    if (!is_mus) { mx = 0.f; mlo = 0.f; mhi = 0.f; mst = 0.f; }
    if (!acts) act = 0.f;
    // diverged walkers (lean_compute): every mass of the walker NaN somewhere in its position, unpinned, with a spring ->
    // finite stand-ins now, NaN state and outputs after the integrator
    bool dead = false;
    {
        const bool nanp = is_mass && (__builtin_isnan(p3[0]) || __builtin_isnan(p3[1]) || __builtin_isnan(p3[2]));
        if (__builtin_expect(__ballot(nanp) != 0ull, 0)) {   // wave-uniform, rare
            const unsigned long long db = __ballot(nanp && pin == 0 && io1 > io0);
            const int mwn = s_mo[mw + 1] - mlm;
            const unsigned long long gm = (mwn >= 64) ? ~0ull : (((1ull << mwn) - 1ull) << mlm);
            dead = is_mass && (db & gm) == gm;
            if (dead) {
                p3[0] = (float)(lane - mlm); p3[1] = 0.f; p3[2] = 0.f;
                v3[0] = 0.f; v3[1] = 0.f; v3[2] = 0.f;
            }
        }
    }
    if (kp.prio) __builtin_amdgcn_s_setprio(0);
    STAMP(1);

    // ================= incidence lists into LDS; act (gym/optimized_walker.py:27-43,164-172)
#pragma unroll
    for (int it = 0; it < NE; it++)
        if (lane + 64 * it < nE) s_inc[lane + 64 * it] = gi[it];
    if (lane == 0) s_inc[nE] = 0u;   // the read-ahead pad after the last list (mass_accumulate_v2)
    float x = mx;
    if (acts) {
        x = (kp.action_mode == 1) ? ((act != 0.f) ? x + mst : x - mst) : x + act;
        if (mlo > x) x = mlo;     // Python max(x, originx*minl)
        if (mhi < x) x = mhi;     // Python min(x, originx*maxl)
        *WG_ST(b.muscle_x, U0 + lane, 1) = x;
    }
    if (is_mus) s_x[lane] = x;
    double ym = recip_m(mf);
    asm volatile("" : "+v"(ym));   // (float)ym stays a conversion, not a float32 division
    wave_sync();
    STAMP(2);

    // ================= springs: gym/engine.py:78-102 + gym/optimized_walker.py:92-106 =================
    bool gtiny = false;   // a damping force of this lane's springs outside the mass loop's exact quotient range
    const bool pos_ok = __all(fexp3(p3[0], p3[1], p3[2]) >= -55);   // (spring_terms)
#pragma unroll
    for (int it = 0; it < NE; it++) {
        if (64 * it >= nE) continue;                       // wave-uniform
        const int le = lane + 64 * it;
        const EdgeRec e = er[it];
        const int ew_w = le < nE ? eww[it] : 0;
        const int elm = s_mo[ew_w], ew = le - s_eo[ew_w], eA = s_uo[ew_w + 1] - s_uo[ew_w];
        const int bi = (elm + edge_i(e.ij)) << 2, bj = (elm + edge_j(e.ij)) << 2;
        const float pix = lane_gather(p3[0], bi), piy = lane_gather(p3[1], bi), piz = lane_gather(p3[2], bi);
        const float pjx = lane_gather(p3[0], bj), pjy = lane_gather(p3[1], bj), pjz = lane_gather(p3[2], bj);
        const float vix = lane_gather(v3[0], bi), viy = lane_gather(v3[1], bi), viz = lane_gather(v3[2], bi);
        const float vjx = lane_gather(v3[0], bj), vjy = lane_gather(v3[1], bj), vjz = lane_gather(v3[2], bj);
        const bool mus = le < nE && ew < eA;
        const float xs = s_x[mus ? s_uo[ew_w] + ew : 0];
        const float xr = mus ? xs : e.rest;
        if (le < nE) {
            if (WG_ABLATE & 1)   // profiling builds only: no spring arithmetic
                ts.put(le, xr + pix + pjx + vix + vjx, piy + pjy + viy + vjy, piz + pjz + viz + vjz, e.k, e.c, 0.f);
            else
                spring_edge_regs(e, le, xr, pix, piy, piz, pjx, pjy, pjz, vix, viy, viz, vjx, vjy, vjz, ts, 0, gtiny,
                                 pos_ok);
        }
    }
    wave_sync();
    // any spring of the wave with a damping force outside the exact range: every mass loop of the wave divides by m with
    // IEEE divisions (rare: damping forces below 2^-80)
    const bool wave_tiny = __any(gtiny);
    STAMP(3);

    // ================= masses: ordered accumulation, env forces, Point.run1 =================
    EnvTerms et{};
    et = env_terms(kp, mf, (float)ym, v3[0], v3[1], v3[2]);   // (as the lean kernel)
    float px = 0.f, py = 0.f, pz = 0.f, vx = 0.f, vy = 0.f, vz = 0.f, ax = 0.f, ay = 0.f, az = 0.f;
    bool hit = false;
    if (is_mass) {
        mass_accumulate_v2(ts, reinterpret_cast<const uint16_t *>(s_inc) + 2 * mlb, mlb, io0,
                           (WG_ABLATE & 2) ? min(io1, io0 + 1) : io1, mf, ym, ax, ay, az, wave_tiny);
        mass_tail(kp, mf, (float)ym, p3, v3, px, py, pz, vx, vy, vz, ax, ay, az, hit, pin != 0, &et);
        if (dead) {
            px = __builtin_nanf(""); py = px; pz = px; vx = px; vy = px; vz = px; ax = px; ay = px; az = px;
            hit = false;
        }
        const uint32_t pl = (uint32_t)(P0 + lane);
        float *gpo = WG_ST(b.pos, pl, 3), *gvo = WG_ST(b.vel, pl, 3), *gao = WG_ST(b.acc, pl, 3);
        gpo[0] = px; gpo[1] = py; gpo[2] = pz;
        gvo[0] = vx; gvo[1] = vy; gvo[2] = vz;
        gao[0] = ax; gao[1] = ay; gao[2] = az;
        if (b.contact) at_u32w(b.contact, pl) = (uint8_t)hit;
        if (b.radius) b.radius[pl] = hit ? 3.0 : 1.0;   // gym/optimized_env.py:156,175
    }
    STAMP(4);
    // contacts after run1 and the all-stopped test, one bit per mass lane (walker w: lanes [s_mo[w], s_mo[w + 1]))
    const float nvm = is_mass ? np_norm3(vx, vy, vz) : 0.f;
    const unsigned long long hb = __ballot(is_mass && (py - kp.ground < 0.f));
    const unsigned long long sb = __ballot(is_mass && nvm < 0.1f);
    wave_sync();                       // every lane is done reading the spring terms: their region takes the
    if (is_mass) {                     // per-mass reduction terms, the damping region the walker partials
        const float nv = nvm;
        s_tp[3 * lane] = px; s_tp[3 * lane + 1] = py; s_tp[3 * lane + 2] = pz;
        s_tn[lane] = nv;
        s_tk[lane] = dead ? nv : mf * np_sq(nv);   // p.m * norm(p.v) ** 2 (gym/optimized_env.py:242)
        s_te[lane] = (float)((double)mf * kp.g) * (py - kp.ground);
    }
    wave_sync();

    // ================= per-walker reductions, 8 lanes per walker (numpy's summation orders) ==========
    // r 0-2: sequential sums of pos[:, r] (getstat mid / info centroid); r 3: pairwise y (np.mean);
    // r 4-6: pairwise |v|, m|v|^2, m*g*(y - ground); r 7: contact count << 1 | all-stopped, from the ballots
    for (int idx = lane; idx < ((WG_ABLATE & 32) ? 0 : nw * 8); idx += 64) {   // (ablation bit 32: no reductions)
        const int w = idx >> 3, r = idx & 7;
        const int lm = s_mo[w], M = s_mo[w + 1] - lm;
        float v;
        if (r == 7) {
            const unsigned long long wm = (M == 64) ? ~0ull : (((1ull << M) - 1ull) << lm);
            v = __int_as_float((__popcll(hb & wm) << 1) | ((sb & wm) == wm ? 1 : 0));
        } else {
            // every lane runs both sums (one path): lanes 0-2 keep the sequential one, 3-6 the pairwise one
            const float *src = r == 3 ? s_tp + 3 * lm + 1 : r == 5 ? s_tk + lm : r == 6 ? s_te + lm : s_tn + lm;
            float vs, vp;
            dual_sum_lds(s_tp + 3 * lm + (r < 3 ? r : 0), 3, src, r == 3 ? 3 : 1, M, vs, vp);
            v = r < 3 ? vs : vp;
        }
        s_red[idx] = v;
    }
    wave_sync();
    if (lane < nw) {
        const int M = s_mo[lane + 1] - s_mo[lane];
        const float fM = (float)M;
        const double yM = rcp64_nr((double)M);
        const float *rd = s_red + 8 * lane;
        const float cy = fdiv_count(rd[3], fM, yM);
        const int packed = __float_as_int(rd[7]);
        const int hits = packed >> 1, all = packed & 1;
        const int steps = wsteps + 1;
        *WG_ST(b.steps, w0 + lane, 1) = steps;
        if (o.steps) *WG_ST(o.steps, wrow, 1) = steps;
        if (o.reward) *WG_ST(o.reward, wrow, 1) = (cy + (-fdiv_count(rd[4], fM, yM)) * 0.1f) + neg_half_count(hits);
        if (o.done) {
            int done = steps >= kp.max_steps;
            if (!done && cy < kp.done_y) done = 1;
            if (!done && steps > 100) done = all;
            at_u32w(o.done, (uint32_t)wrow) = (uint8_t)done;
        }
        // the walker's mean position (np.mean: info's centroid, getstat's mid), once per walker: every mass lane of the
        // observation rows reads it from LDS instead of dividing again (-25 VALU per wave)
        const float mx = fdiv_count(rd[0], fM, yM), my = fdiv_count(rd[1], fM, yM), mz = fdiv_count(rd[2], fM, yM);
        s_mid[3 * lane] = mx; s_mid[3 * lane + 1] = my; s_mid[3 * lane + 2] = mz;
        if (o.centroid) {
            float *c = WG_ST(o.centroid, wrow, 3);
            c[0] = mx; c[1] = my; c[2] = mz;
        }
        if (o.energy) *WG_ST(o.energy, wrow, 1) = 0.5f * rd[5] + rd[6];
    }
    wave_sync();
    STAMP(5);

    // ================= observation rows: Creature.getstat (gym/optimized_walker.py:129-162) =========
    // Walker w's row (the caller's row s_row[w]) is per*M_w values, the 3 conmid values, A_w muscle lengths, then
    // zeros to the stride.  Each mass lane stores its 3d values straight from registers as d-float pieces, each
    // muscle lane its length; the padding is written only when the caller's buffer is not known to be clean.
    if (o.obs && !(WG_ABLATE & 16)) {
        constexpr int d = IN3D ? 3 : 2, per = 3 * d;
        const int stride = o.obs_stride, nmid = kp.conmid ? 3 : 0;
        typedef float fvd __attribute__((ext_vector_type(d), aligned(4)));
        if (is_mass) {
            const float *rd = kp.midform == 2 ? s_red + 8 * mw : s_mid + 3 * mw;   // G1 getstat: the SUM; else the mean
            float *dst = WG_ST(o.obs, (uint32_t)s_row[mw] * (uint32_t)stride + per * (lane - mlm), 1);
            const float pm[3] = {px, py, pz}, vm[3] = {vx, vy, vz}, am[3] = {ax, ay, az};
            fvd vp, vv, va;
#pragma unroll
            for (int c = 0; c < d; c++) {
                const float mid = rd[c];
                vp[c] = kp.midform ? (pm[c] - mid) * kp.pk : pm[c] * kp.pk;
                vv[c] = vm[c] * kp.vk;
                va[c] = am[c] * kp.ak;
            }
            *reinterpret_cast<fvd *>(dst) = vp;        // (a 3-vector's type is 16 B: no array indexing over fvd)
            *reinterpret_cast<fvd *>(dst + d) = vv;
            *reinterpret_cast<fvd *>(dst + 2 * d) = va;
        }
        if (lane < nw && nmid) {
            const int M = s_mo[lane + 1] - s_mo[lane];
            float *row = WG_ST(o.obs, (uint32_t)wrow * (uint32_t)stride + per * M, 1);
            const float *rd = s_red + 8 * lane;
            for (int c = 0; c < 3; c++) row[c] = kp.midform == 2 ? rd[c] : kp.midform ? rd[c] / (float)M : 0.f;
        }
        if (is_mus)
            *WG_ST(o.obs, (uint32_t)s_row[uw] * (uint32_t)stride + per * (s_mo[uw + 1] - s_mo[uw]) + nmid + ua, 1) =
                x * kp.mk;
        if (!o.obs_pad_clean) {
            // zeros from each row's own length to the stride; row w = i / stride
            const float inv = 1.f / (float)stride;
            for (int i = lane; i < nw * stride; i += 64) {
                const int w = fdiv(i, stride, inv), c = i - w * stride;
                const int len = per * (s_mo[w + 1] - s_mo[w]) + nmid + (s_uo[w + 1] - s_uo[w]);
                if (c >= len) *WG_ST(o.obs, (uint32_t)s_row[w] * (uint32_t)stride + c, 1) = 0.f;
            }
        }
    }
    STAMP(6);
#ifdef WG_STAMPS
    if (lane == 0 && stamp_wave < (1 << 16)) {   // slot 7: HW_ID (gfx9 hwreg 4) | XCC_ID (gfx940+ hwreg 20) << 32
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        g_stamps[stamp_wave * 8 + 7] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
    }
#endif
}

// reset: v += noise, steps = 0 (PhysicsEnv.reset, gym/optimized_env.py:53-68).  zmode 0: x, y (2D);
// 1: x, y, z (in3d); 2: every component whose noise is not exactly +0.0 (wg_reset_noise)
__global__ void walker_reset_kernel(wg_batch b, const float *__restrict__ noise, const uint8_t *__restrict__ mask,
                                    int zmode) {
    const int P = b.ragged ? b.mass_off[b.N] : b.N * b.M;
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < P; q += gridDim.x * blockDim.x) {
        int w;
        if (b.ragged) {
            int lo = 0, hi = b.N - 1;
            while (lo < hi) { const int mid = (lo + hi + 1) >> 1; if (b.mass_off[mid] <= q) lo = mid; else hi = mid - 1; }
            w = lo;
        } else {
            w = q / b.M;
        }
        if (mask && !mask[w]) continue;
        if (noise) {
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const float n = noise[3 * q + c];
                const bool add = zmode == 2 ? __float_as_uint(n) != 0u : (c < 2 || zmode == 1);
                if (add) b.vel[3 * q + c] = b.vel[3 * q + c] + n;
            }
        }
    }
    for (int w = blockIdx.x * blockDim.x + threadIdx.x; w < b.N; w += gridDim.x * blockDim.x)
        if (!mask || mask[w]) b.steps[w] = 0;
}

// Opt-in per-walker info of the state after a step or observe (wg_outputs.nonfinite / momentum, ABI 10): one lane
// per walker walks its masses in point order.  nonfinite: any pos / vel / acc component inf or NaN (SURVEY §5 failure
// detection; done is untouched).  momentum: Point.momentum (gym/engine.py:160-166), m_sum = float32 zeros, then
// m_sum += v * m point by point (v float32, m the point's mass: numpy's float32 product, then a float32 add).
// Outputs at the caller's row (wg_batch.row).  Not on the headline path: a caller that asks for neither pays nothing.
// A ragged batch's walker range is its plan slice [plan[0], plan[plan_blocks]) (the other ranges of a wg_step_ranges
// call may still be stepping theirs).
__global__ __launch_bounds__(256) void walker_info_kernel(wg_batch b, uint8_t *__restrict__ nonfinite,
                                                          float *__restrict__ momentum, const int32_t *__restrict__ plan,
                                                          int plan_blocks) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= b.N) return;
    if (plan && (w < plan[0] || w >= plan[plan_blocks])) return;
    const int p0 = b.ragged ? b.mass_off[w] : w * b.M, p1 = b.ragged ? b.mass_off[w + 1] : p0 + b.M;
    float mx = 0.f, my = 0.f, mz = 0.f;
    bool bad = false;
    for (int q = p0; q < p1; q++) {
        const float *pv = b.pos + 3 * (size_t)q, *vv = b.vel + 3 * (size_t)q, *av = b.acc + 3 * (size_t)q;
        const float vx = vv[0], vy = vv[1], vz = vv[2], m = b.mass[q];
        bad = bad || !(__builtin_isfinite(pv[0]) && __builtin_isfinite(pv[1]) && __builtin_isfinite(pv[2]) &&
                       __builtin_isfinite(vx) && __builtin_isfinite(vy) && __builtin_isfinite(vz) &&
                       __builtin_isfinite(av[0]) && __builtin_isfinite(av[1]) && __builtin_isfinite(av[2]));
        mx = mx + vx * m; my = my + vy * m; mz = mz + vz * m;
    }
    const int r = caller_row(b, w);
    if (nonfinite) nonfinite[r] = (uint8_t)bad;
    if (momentum) { momentum[3 * r] = mx; momentum[3 * r + 1] = my; momentum[3 * r + 2] = mz; }
}

// ------------------------------------------------------------------ host side
int env_int(const char *name, int dflt);
int wave_passes(int M, int K);

KParams make_kparams(const wg_params &p) {
    KParams k;
    k.neg_g = (float)(-p.g);
    k.neg_dampk = (float)(-p.dampk);
    k.ground = (float)p.ground;
    k.neg_groundk = (float)(-p.groundk);
    k.neg_grounddamp = (float)(-p.grounddamp);
    k.friction = (float)p.friction;
    k.dt = (float)p.dt;
    k.pk = (float)p.pk; k.vk = (float)p.vk; k.ak = (float)p.ak; k.mk = (float)p.mk;
    k.done_y = (float)(p.ground - 50.0);
    k.g = p.g;
    k.max_steps = p.max_steps; k.midform = p.midform; k.conmid = p.conmid;
    k.spring_mode = p.spring_mode; k.action_mode = p.action_mode;
    k.integrator = p.integrator;
    k.pair_mode = p.pair_mode;
    k.pair_g = p.pair_g;
    k.pair_k = p.pair_k;
    k.pair_e = p.pair_e;
    k.bounce_kh = (float)(p.bounce_k / 2);
    for (int i = 0; i < 3; i++) k.g3g[i] = (float)p.g3_gravity[i];
    k.g3_damp = (float)p.g3_damping;
    k.g3_dragc = (float)(-0.5 * p.g3_air);
    k.g3_level = (float)p.g3_ground_level;
    k.g3_rest = (float)p.g3_restitution;
    k.g3_fric = (float)p.g3_friction;
    k.g3_ground = p.g3_ground;
    k.friction_mode = p.friction_mode;
    k.prio = env_int("WG_LEAN_PRIO", 1);
    k.xcd = env_int("WG_XCD", 3);   // both kernels (profiles/r03e_ab_canon.json, r03d_ab_ragged_window_xcd.json)

    k.dt2 = (float)(p.dt * p.dt);
    return k;
}

constexpr int RAG_P = 256, RAG_E = 512, RAG_U = 256, RAG_W = 64;
constexpr int LDS_LIMIT = 160 * 1024;

int validate(const wg_batch *b) {
    if (!b) return fail(WG_EINVAL, "null batch");
    if (b->N < 0 || b->M < 1 || b->K < 0 || b->A < 0 || b->A > b->K)
        return fail(WG_EINVAL, "bad sizes N=%d M=%d K=%d A=%d", b->N, b->M, b->K, b->A);
    if (2 * b->K > 65535) return fail(WG_ERANGE, "K=%d exceeds the u16 incidence encoding", b->K);
    if (b->M > WG_MAX_M) return fail(WG_ERANGE, "M=%d > %d masses per walker", b->M, WG_MAX_M);
    if (!b->pos || !b->vel || !b->acc || !b->mass || !b->steps || !b->muscle_x)
        return fail(WG_EINVAL, "missing state pointer");
    if (b->K > 0 && (!b->edges || !b->inc || !b->inc_off)) return fail(WG_EINVAL, "missing edge pointer");
    if (b->M > 32767) return fail(WG_ERANGE, "M=%d exceeds the 15-bit edge endpoint encoding", b->M);
    if (!b->inc_off) return fail(WG_EINVAL, "missing inc_off");
    if (b->ragged < 0 || b->ragged > 2) return fail(WG_EINVAL, "ragged must be 0, 1 or 2");
    if (b->ragged && (!b->mass_off || !b->edge_off || !b->muscle_off))
        return fail(WG_EINVAL, "ragged batch without offsets");
    if (!b->ragged && b->row) return fail(WG_EINVAL, "row (a walker permutation) is for ragged batches only");
    if (b->ragged == 2 && !wave_passes(b->M, b->K))
        return fail(WG_EINVAL, "ragged = 2 (wave tiles) needs M <= 64 and at most 8 spring passes (M=%d K=%d)", b->M, b->K);
    return 0;
}

Geo uniform_geo(const wg_batch *b, int obs_stride, bool no_lite = false) {
    Geo g{};
    // walkers per workgroup: fill the 256 mass lanes, keep edges within EPL registers per lane,
    // and make sure the grid has >= 512 workgroups when the batch allows it.
    int W = std::max(1, NTHREADS / b->M);
    if (b->M > 64 && env_int("WG_WIDE", 1)) {
        // M > 64: the workgroup size (256..512 threads) that leaves the fewest idle lanes; 100-mass chains run
        // 5 walkers on 512 threads (98 % of the lanes busy) instead of 2 on 256 (78 %)
        int best = 0, bestT = NTHREADS;
        for (int T = NTHREADS; T <= MAXT; T += 64) {
            const int w = T / b->M;
            if (w >= 1 && (int64_t)w * b->M * bestT > (int64_t)best * T) { best = w * b->M; bestT = T; W = w; }
        }
    }
    if (b->K > 0) W = std::max(1, std::min(W, EPL * MAXT / std::max(1, b->K)));
    while (W > 1 && (b->N + W - 1) / W < 512) W = std::max(1, W / 2);
    g.W = W;
    const bool shfl_shape = b->M <= 64 && (64 % b->M) == 0 && !(WG_ABLATE & 64);
    for (;;) {
        g.Pcap = g.W * b->M; g.Ecap = g.W * b->K; g.Ucap = g.W * b->A;
        g.tbytes = std::max(g.Ecap * 3 * 8, g.W * std::max(0, obs_stride) * 4);
        g.lite = (shfl_shape && g.W * b->M <= MAXT && !no_lite) ? 1 : 0;   // pair passes need the LDS copies
        g.threads = std::min(MAXT, std::max(64, ((g.W * b->M + 63) / 64) * 64));
        if (b->K > 0 && g.W * b->K > EPL * g.threads) g.threads = MAXT;
        g.lds = carve_bytes(g);
        if (g.lds <= 64 * 1024 || g.W == 1) break;
        g.W = std::max(1, g.W / 2);
    }
    g.invM = 1.f / (float)b->M;
    g.invK = 1.f / (float)std::max(1, b->K);
    g.invA = 1.f / (float)std::max(1, b->A);
    return g;
}

Geo ragged_geo(const wg_batch *b) {
    Geo g{};
    g.threads = NTHREADS;
    g.W = RAG_W;
    g.Pcap = std::max(RAG_P, b->M);
    g.Ecap = std::max(RAG_E, b->K);
    g.Ucap = std::max(RAG_U, b->A);
    g.tbytes = g.Ecap * 3 * 8;
    g.lite = 0;
    g.lds = carve_bytes(g);
    g.invM = g.invK = g.invA = 0.f;
    return g;
}

template <bool STEP, bool RAGGED, bool IN3D, int PWD, bool SHFL>
int launch(const wg_batch *b, const KParams &kp, const float *action, int cols, int astride,
           const wg_outputs &o, const int32_t *plan, int blocks, const Geo &g, hipStream_t stream) {
    // (+ the static 512 B of the powf tables in LDS)
    const int lds_static = (int)(sizeof(s_pw_log2) + sizeof(s_pw_exp2));
    if (g.lds + lds_static > LDS_LIMIT)
        return fail(WG_ERANGE, "workgroup needs %d B of LDS (> 160 KiB)", g.lds + lds_static);
    WG_KLAUNCH((walker_step_kernel<STEP, RAGGED, IN3D, PWD, SHFL>), dim3(blocks), dim3(g.threads), (uint32_t)g.lds, stream,
               *b, kp, action, cols, astride, kout(o), plan, g);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(WG_EHIP, "launch failed: %s", hipGetErrorString(e));
    return 0;
}

// register (shuffle) reductions: every walker's masses are adjacent lanes of one wave
bool shfl_ok(const wg_batch *b, const Geo &g) { return !b->ragged && g.lite; }

template <bool STEP, int PWD>
int dispatch2(const wg_batch *b, const KParams &kp, bool in3d, const float *a, int cols, int astride,
              const wg_outputs &o, const int32_t *plan, int blocks, const Geo &g, hipStream_t st) {
    if (b->ragged) {
        return in3d ? launch<STEP, true, true, PWD, false>(b, kp, a, cols, astride, o, plan, blocks, g, st)
                    : launch<STEP, true, false, PWD, false>(b, kp, a, cols, astride, o, plan, blocks, g, st);
    }
    if (PWD == 0 && shfl_ok(b, g)) {
        return in3d ? launch<STEP, false, true, 0, true>(b, kp, a, cols, astride, o, plan, blocks, g, st)
                    : launch<STEP, false, false, 0, true>(b, kp, a, cols, astride, o, plan, blocks, g, st);
    }
    return in3d ? launch<STEP, false, true, PWD, false>(b, kp, a, cols, astride, o, plan, blocks, g, st)
                : launch<STEP, false, false, PWD, false>(b, kp, a, cols, astride, o, plan, blocks, g, st);
}
// ---- lean kernel selection: uniform batch, M | 64 with M >= 4, the wave's edges in <= 8 register
// passes, its muscles in one pass, and a workgroup LDS footprint that keeps >= 2 workgroups per CU.
// Knobs (read on every call, so one process can A/B them): WG_LEAN=0 selects the barrier kernels;
// WG_LEAN_WAVES 1/2/4 waves per workgroup; WG_LEAN_PRIO 0/1 load-phase priority.
int env_int(const char *name, int dflt) {
    const char *e = getenv(name);
    return (e && *e) ? atoi(e) : dflt;
}

bool lean_enabled() { return env_int("WG_LEAN", 1) != 0; }

// The barrier-free kernels address their loads as SGPR base + 32-bit byte offset (at_u32): every array of the batch
// must then span less than 4 GiB (positions 12 B and spring records 16 B per element dominate; M, K are maxima).
bool u32_bytes(const wg_batch *b) {
    const int64_t lim = 1ll << 32;
    return (int64_t)b->N * b->M * 12 < lim && (int64_t)b->N * b->K * 16 < lim && (int64_t)b->N * b->A * 8 < lim &&
           (int64_t)b->N * (b->M + 1) * 2 < lim;
}
// and their observation rows as 32-bit byte offsets (WG_ST)
bool obs_u32(const wg_batch *b, int obs_stride) { return (int64_t)b->N * std::max(obs_stride, 1) * 4 < (1ll << 32); }

bool lean_geo(const wg_batch *b, int obs_stride, LeanGeo *out, int spring_mode = 0) {
    const int M = b->M;
    if (b->ragged || M < 4 || M > 64 || (64 % M) != 0 || b->K < 1 || !lean_enabled() || (WG_ABLATE & 128)) return false;
    if (spring_mode != 0) return false;          // the G2-compat element runs on the workgroup kernel
    // 32-bit element offsets inside the kernel, 32-bit byte offsets for its loads (at_u32)
    if ((int64_t)b->N * b->M * 3 >= (1ll << 31) || (int64_t)b->N * b->K * 4 >= (1ll << 31) ||
        !obs_u32(b, obs_stride) || !u32_bytes(b))
        return false;
    LeanGeo g{};
    g.wpw = 64 / M;
    // small batches: fewer walkers per wave until there are 512 wave tiles (two per CU), so a latency-bound step
    // spreads over more waves (4,096 Balance-v0 walkers: 16 -> 8 walkers per wave, 6.40 -> 5.97 us per step,
    // profiles/r02_ab_balance4096_wpw.json); WG_LEAN_WPW (experiment) caps the count
    while (g.wpw > 1 && (b->N + g.wpw - 1) / g.wpw < 512) g.wpw >>= 1;
    const int wcap = env_int("WG_LEAN_WPW", 0);
    if (wcap > 0 && wcap < g.wpw) g.wpw = wcap;
    g.lgM = 0;
    while ((1 << g.lgM) < M) g.lgM++;
    if ((g.wpw * b->K + 63) / 64 > 8 || g.wpw * b->A > 64) return false;
    // waves per workgroup: 4 (one workgroup per four tiles) unless the batch has no more tiles than the chip has SIMDs,
    // where one wave per workgroup spreads the latency-bound step over twice the CUs (4,096 Balance-v0 walkers: 5.45
    // against 5.60 us, 65,536 canonical: 44.31 against 44.01; profiles/r04m_ab_*_wpb.json); WG_LEAN_WAVES overrides
    const int wpb = env_int("WG_LEAN_WAVES", 0);
    g.wpb = (wpb == 1 || wpb == 2 || wpb == 4) ? wpb : ((b->N + g.wpw - 1) / g.wpw <= 1024 ? 1 : 4);
    const int ew = g.wpw * b->K;                          // springs of a full wave tile
    g.pl = (ew + 3) & ~3;                                 // spring-term slots: 16-B aligned regions
    // t (f64 x3) | df (f32 x3) | incidence words | x (observation rows go from registers to HBM, no LDS tile)
    g.off_df = align16(g.pl * 24);
    g.off_inc = g.off_df + align16(g.pl * 12);
    g.off_x = g.off_inc + align16(ew * 4 + 4);              // + the zero word after the last list (mass_accumulate_v2)
    g.slice = g.off_x + align16(std::max(1, g.wpw * b->A) * 4);
    if (4 * g.slice > 80 * 1024) return false;
    g.invK = 1.f / (float)b->K;
    g.invA = 1.f / (float)std::max(1, b->A);
    g.invM = 1.f / (float)M;
    g.nblk = (b->N + g.wpb * g.wpw - 1) / (g.wpb * g.wpw);   // = lean_blocks
    *out = g;
    return true;
}

// grid of a lean launch: one tile (64 / M walkers) per wave
int lean_blocks(const wg_batch *b, const LeanGeo &g) { return (b->N + g.wpb * g.wpw - 1) / (g.wpb * g.wpw); }

int launch_lean(const wg_batch *b, const KParams &kp, bool in3d, const float *a, int cols, int astride,
                const wg_outputs &o, const LeanGeo &g, hipStream_t st) {
    const int blocks = lean_blocks(b, g);
    const int ne = (g.wpw * b->K + 63) / 64;
    // WG_LDS_PAD (diagnostic): extra LDS bytes per workgroup, to measure the kernel at lower occupancy
    const int lds = g.wpb * g.slice + std::max(0, env_int("WG_LDS_PAD", 0));
#define WG_LAUNCH_LEAN(D3, NE_)                                                                                  \
    WG_KLAUNCH((walker_step_lean<D3, NE_>), dim3(blocks), dim3(64 * g.wpb), (uint32_t)lds, st, *b, kp, a, cols,  \
               astride, kout(o), g)
#define WG_LEAN_NE(D3)                                                         \
    do {                                                                       \
        if (ne == 2) WG_LAUNCH_LEAN(D3, 2);                                    \
        else if (ne == 3) WG_LAUNCH_LEAN(D3, 3);                               \
        else if (ne == 4) WG_LAUNCH_LEAN(D3, 4);                               \
        else WG_LAUNCH_LEAN(D3, 8);                                            \
    } while (0)
    if (ne <= 1) {   // (the NE = 1 entry with preloaded arguments)
        if (in3d)
            WG_KLAUNCH((walker_step_lean1<true>), dim3(blocks), dim3(64 * g.wpb), (uint32_t)lds, st, b->pos, b->vel,
                               b->edges, b->inc, b->N, b->M, b->K, g.wpw, g.wpb, (int)((unsigned)g.nblk | ((unsigned)(kp.xcd & 2) << 29) | ((unsigned)(kp.prio != 0) << 31)), *b,
                               kp, a, cols, astride, kout(o), g);
        else
            WG_KLAUNCH((walker_step_lean1<false>), dim3(blocks), dim3(64 * g.wpb), (uint32_t)lds, st, b->pos, b->vel,
                               b->edges, b->inc, b->N, b->M, b->K, g.wpw, g.wpb, (int)((unsigned)g.nblk | ((unsigned)(kp.xcd & 2) << 29) | ((unsigned)(kp.prio != 0) << 31)), *b,
                               kp, a, cols, astride, kout(o), g);
    } else if (in3d) {
        WG_LEAN_NE(true);
    } else {
        WG_LEAN_NE(false);
    }
#undef WG_LEAN_NE
#undef WG_LAUNCH_LEAN
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(WG_EHIP, "launch failed: %s", hipGetErrorString(e));
    return 0;
}

int launch_lean_rollout(const wg_batch *b, const KParams &kp, bool in3d, const float *a, int cols, int astride,
                        int64_t astep, const wg_outputs &o, int n_steps, const LeanGeo &g, hipStream_t st) {
    const int blocks = lean_blocks(b, g);
    const int ne = (g.wpw * b->K + 63) / 64;
    const int lds = g.wpb * g.slice;
#define WG_LAUNCH_RO(D3, NE_)                                                                                    \
    hipLaunchKernelGGL((walker_rollout_lean<D3, NE_>), dim3(blocks), dim3(64 * g.wpb), lds, st, *b, kp, a, cols, \
                       astride, astep, kout(o), n_steps, g)
#define WG_RO_NE(D3)                                                                                             \
    do {                                                                                                         \
        if (ne <= 1) WG_LAUNCH_RO(D3, 1);                                                                        \
        else if (ne == 2) WG_LAUNCH_RO(D3, 2);                                                                   \
        else if (ne == 3) WG_LAUNCH_RO(D3, 3);                                                                   \
        else if (ne == 4) WG_LAUNCH_RO(D3, 4);                                                                   \
        else WG_LAUNCH_RO(D3, 8);                                                                                \
    } while (0)
    if (in3d) WG_RO_NE(true); else WG_RO_NE(false);
#undef WG_RO_NE
#undef WG_LAUNCH_RO
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(WG_EHIP, "launch failed: %s", hipGetErrorString(e));
    return 0;
}

// ---- ragged wave kernel (wg_batch.ragged = 2): spring passes, planner, geometry, launch
// Spring passes of a wave tile from the batch maxima: enough for the longest walker, and for 64 masses of the
// densest one (K / M springs per mass), rounded up to an instantiated NE (1, 2, 3, 4, 8); 0 = not eligible.
int wave_passes(int M, int K) {
    if (M < 1 || M > 64 || K < 0) return 0;
    int ne = std::max((K + 63) / 64, (K + M - 1) / M);
    ne = std::max(ne, 1);
    if (ne > 8) return 0;
    return ne <= 4 ? ne : 8;
}

bool rag_geo(const wg_batch *b, int obs_stride, RagGeo *out) {
    const int ne = wave_passes(b->M, b->K);
    if (b->ragged != 2 || ne == 0 || b->A > 64 || !u32_bytes(b) || !obs_u32(b, obs_stride)) return false;
    RagGeo g{};
    const int wpb = env_int("WG_LEAN_WAVES", 4);
    g.wpb = (wpb == 1 || wpb == 2) ? wpb : 4;
    const int ec = 64 * ne;                                      // spring slots of a tile
    // spring terms t (f64 x3), later the per-mass reduction terms | damping forces df, later the walker partials |
    // incidence words | muscle x | walker offsets and rows
    g.off_df = align16(std::max(ec * 24, 4 * 64 * 6));
    g.off_inc = g.off_df + align16(std::max(ec * 12, 4 * RW_MAXW * 8));
    g.off_x = g.off_inc + align16(ec * 4 + 4);                   // + the read-ahead pad word (mass_accumulate_v2)
    g.off_wo = g.off_x + align16(64 * 4);
    g.slice = g.off_wo + align16(4 * (RW_MAXW + 1) * 3 + 4 * RW_MAXW + 12 * RW_MAXW);   // + the walkers' means
    *out = g;
    return true;
}

int launch_waves(const wg_batch *b, const KParams &kp, bool in3d, const float *a, int cols, int astride,
                 const wg_outputs &o, const int32_t *plan, int ntiles, const RagGeo &g, hipStream_t st) {
    const int ne = wave_passes(b->M, b->K);
    const int blocks = (ntiles + g.wpb - 1) / g.wpb;
    const int lds = g.wpb * g.slice;
#define WG_LAUNCH_WAVES(D3, NE_)                                                                                  \
    WG_KLAUNCH((walker_step_waves<D3, NE_>), dim3(blocks), dim3(64 * g.wpb), (uint32_t)lds, st, *b, kp, a, cols,   \
               astride, kout(o), plan, ntiles, g)
#define WG_WAVES_NE(D3)                                                        \
    do {                                                                       \
        if (ne <= 1) WG_LAUNCH_WAVES(D3, 1);                                   \
        else if (ne == 2) WG_LAUNCH_WAVES(D3, 2);                              \
        else if (ne == 3) WG_LAUNCH_WAVES(D3, 3);                              \
        else if (ne == 4) WG_LAUNCH_WAVES(D3, 4);                              \
        else WG_LAUNCH_WAVES(D3, 8);                                           \
    } while (0)
    if (in3d) WG_WAVES_NE(true); else WG_WAVES_NE(false);
#undef WG_WAVES_NE
#undef WG_LAUNCH_WAVES
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(WG_EHIP, "launch failed: %s", hipGetErrorString(e));
    return 0;
}

int reset_impl(const wg_batch *b, const float *noise, const uint8_t *mask, int zmode, hipStream_t stream) {
    int rc = validate(b);
    if (rc) return rc;
    if (b->N == 0) return 0;
    const long P = b->ragged ? -1 : (long)b->N * b->M;
    const int blocks = P > 0 ? (int)std::min<long>((P + 255) / 256, 4096) : 1024;
    hipLaunchKernelGGL(walker_reset_kernel, dim3(blocks), dim3(256), 0, stream, *b, noise, mask, zmode);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(WG_EHIP, "reset launch failed: %s", hipGetErrorString(e));
    return 0;
}

template <bool STEP>
int dispatch(const wg_batch *b, const KParams &kp, bool in3d, const float *a, int cols, int astride,
             const wg_outputs &o, const int32_t *plan, int blocks, const Geo &g, hipStream_t st) {
    return b->M <= 128 ? dispatch2<STEP, 0>(b, kp, in3d, a, cols, astride, o, plan, blocks, g, st)
                       : dispatch2<STEP, 3>(b, kp, in3d, a, cols, astride, o, plan, blocks, g, st);
}

int run(const wg_batch *b, const wg_params *p, const float *action, int32_t cols, int32_t astride,
        int64_t astep, const wg_outputs *o, int32_t n_steps, const int32_t *plan, int32_t plan_blocks,
        hipStream_t stream, bool step, bool resident = false, bool check_only = false, int s_first = 0) {
    int rc = validate(b);
    if (rc) return rc;
    if (!p) return fail(WG_EINVAL, "null params");
    if (b->N == 0 || n_steps <= 0) return 0;
    if (action && (cols < 0 || astride < cols)) return fail(WG_EINVAL, "bad action stride");
    if (action && p->action_mode == 1 && !b->muscle_stride) return fail(WG_EINVAL, "discrete actions need muscle_stride");
    if (p->integrator < 0 || p->integrator > 2) return fail(WG_EINVAL, "integrator must be 0/1 (run1) or 2 (run2)");
    if (action && !b->muscle_bounds) return fail(WG_EINVAL, "actions need muscle_bounds");
    if (b->ragged && (!plan || plan_blocks <= 0)) return fail(WG_EINVAL, "ragged batch needs a plan");
    wg_outputs out = o ? *o : wg_outputs{};
    if (out.obs && out.obs_stride <= 0) return fail(WG_EINVAL, "obs_stride must be > 0");
    const KParams kp = make_kparams(*p);
    const Geo g = b->ragged ? ragged_geo(b) : uniform_geo(b, out.obs ? out.obs_stride : 0, step && p->pair_mode != 0);
    if (g.W > g.threads) return fail(WG_ERANGE, "more than %d walkers per workgroup", g.threads);
    const int blocks = b->ragged ? plan_blocks : (b->N + g.W - 1) / g.W;
    LeanGeo lg{};
    const bool act_u32 = !action || (int64_t)b->N * astride * 4 < (1ll << 32);   // at_u32 action offsets
    const bool use_lean = step && act_u32 && lean_geo(b, out.obs ? out.obs_stride : 0, &lg, p->spring_mode);
    RagGeo rgeo{};
    const bool use_waves = step && act_u32 && p->spring_mode == 0 && p->pair_mode == 0 && lean_enabled() &&
                           rag_geo(b, out.obs ? out.obs_stride : 0, &rgeo);
    if (p->spring_mode < 0 || p->spring_mode > 2)
        return fail(WG_EINVAL, "spring_mode %d: 0 (engine.py), 1 (G2 element), 2 (G3 engine) only", p->spring_mode);
    if (step && (p->pair_mode & ~31))
        return fail(WG_EINVAL, "pair_mode %d: bits 1 (gravity), 2 (coulomb), 4 (bounce), 8 (G2 gravity_vec), "
                               "16 (electrostatic) only", p->pair_mode);
    if (step && p->pair_mode != 0 && p->spring_mode != 0)
        return fail(WG_EINVAL, "pair_mode %d needs spring_mode 0", p->pair_mode);
    if (step && (p->pair_mode & 4) && !b->radius)
        return fail(WG_EINVAL, "pair_mode 4 (bounce) needs the radius array");
    if (check_only) return 0;   // wg_step_ranges: every range's arguments checked before any range launches
    const bool extras = out.nonfinite || out.momentum;   // opt-in per-walker info after each step (ABI 10)
    auto info_pass = [&](const wg_outputs &os) -> int {
        if (!(os.nonfinite || os.momentum)) return 0;
        hipLaunchKernelGGL(walker_info_kernel, dim3((b->N + 255) / 256), dim3(256), 0, stream, *b, os.nonfinite,
                           os.momentum, b->ragged ? plan : nullptr, plan_blocks);
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? 0 : fail(WG_EHIP, "info launch failed: %s", hipGetErrorString(e));
    };
    // (the resident rollout keeps the state in registers between steps: with the per-step info extras requested the
    // steps run as per-step launches instead, bit-identical)
    if (resident && use_lean && p->pair_mode == 0 && !extras)   // one launch for every step, state in registers
        return launch_lean_rollout(b, kp, p->in3d != 0, action, cols, astride, action ? astep : 0, out, n_steps, lg,
                                   stream);
    for (int s = s_first; s < s_first + n_steps; s++) {   // (s_first: wg_run_ranges issues one step per call)
        wg_outputs os = out;
        if (os.obs) os.obs += s * os.obs_step;
        if (os.reward) os.reward += s * os.out_step;
        if (os.done) os.done += s * os.out_step;
        if (os.energy) os.energy += s * os.out_step;
        if (os.centroid) os.centroid += 3 * s * os.out_step;
        if (os.steps) os.steps += s * os.out_step;
        if (os.nonfinite) os.nonfinite += s * os.out_step;
        if (os.momentum) os.momentum += 3 * s * os.out_step;
        const float *a = action ? action + s * astep : nullptr;
        if (step && use_lean) rc = launch_lean(b, kp, p->in3d != 0, a, cols, astride, os, lg, stream);
        else if (use_waves) rc = launch_waves(b, kp, p->in3d != 0, a, cols, astride, os, plan, plan_blocks, rgeo, stream);
        else rc = step ? dispatch<true>(b, kp, p->in3d != 0, a, cols, astride, os, plan, blocks, g, stream)
                       : dispatch<false>(b, kp, p->in3d != 0, nullptr, 0, 0, os, plan, blocks, g, stream);
        if (rc) return rc;
        if (extras && (rc = info_pass(os))) return rc;
    }
    return 0;
}

// the launch floor beside a small step (bench.py): an empty launch, and one coalesced load + store per thread
__global__ __launch_bounds__(1024) void floor_empty_kernel(float *) {}
__global__ __launch_bounds__(1024) void floor_load_store_kernel(const float *__restrict__ in, float *__restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    out[i] = in[i] + 1.0f;
}
// mode 2, a device warm-up (bench.py, after RCCL's initialisation has left the GPU idle for seconds): every thread runs
// a dependent chain of float32 FMAs and stores its result (in + chain, so the chain cannot be dropped), ~8 us per launch
// on a full grid at the engine clock; VALU-bound like the step it precedes
__global__ __launch_bounds__(1024) void floor_busy_kernel(const float *__restrict__ in, float *__restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    float x = in[i], y = 0.5f;
#pragma unroll 16
    for (int k = 0; k < 4096; k++) y = __builtin_fmaf(y, 0.99993896484375f, x);
    out[i] = y;
}

}  // namespace

extern "C" {

int wg_abi_version(void) { return WG_ABI_VERSION; }
const char *wg_last_error(void) { return g_err; }

int wg_step(const wg_batch *b, const wg_params *p, const float *action, int32_t action_cols,
            int32_t action_stride, int64_t action_step, const wg_outputs *o, int32_t n_steps,
            const int32_t *plan, int32_t plan_blocks, hipStream_t stream) {
    return run(b, p, action, action_cols, action_stride, action_step, o, n_steps, plan, plan_blocks, stream, true);
}

int wg_rollout(const wg_batch *b, const wg_params *p, const float *action, int32_t action_cols,
               int32_t action_stride, int64_t action_step, const wg_outputs *o, int32_t n_steps,
               const int32_t *plan, int32_t plan_blocks, hipStream_t stream) {
    return run(b, p, action, action_cols, action_stride, action_step, o, n_steps, plan, plan_blocks, stream, true,
               true);
}

int wg_run_ranges(const wg_range *ranges, int32_t n, const wg_params *p, const float *action, int32_t action_cols,
                  int32_t action_stride, int64_t action_step, int32_t n_steps, hipEvent_t *events) {
    if (!ranges || n < 1 || (n > 1 && !events)) return fail(WG_EINVAL, "wg_run_ranges: bad ranges / events");
    // every range checked before the first launch: a bad range fails the call with no walker stepped
    for (int i = 0; i < n; i++) {
        const wg_range &r = ranges[i];
        const int rc = run(r.batch, p, action ? action + r.action_offset : nullptr, action_cols, action_stride,
                           action_step, r.outputs, n_steps, r.plan, r.plan_blocks, r.stream, true, false, true);
        if (rc) return rc;
    }
    if (n_steps <= 0) return 0;
    hipStream_t s0 = ranges[0].stream;
    if (n > 1 && hipEventRecord(events[0], s0) != hipSuccess) return fail(WG_EHIP, "fork event record failed");
    for (int i = 1; i < n; i++)   // (a failed wait leaves nothing issued on the side streams yet: nothing to join)
        if (hipStreamWaitEvent(ranges[i].stream, events[0], 0) != hipSuccess) return fail(WG_EHIP, "fork wait failed");
    // step s of every range is issued before step s + 1 of any: the ranges start together and stay side by side in
    // the hardware queues (range by range, the second range would start only after the host had issued all of the
    // first range's launches).  (Range 0 issued a few steps ahead, or the other ranges started after a timed wait,
    // measured no better: profiles/r04jj_issue_ab.jsonl.)
    auto issue = [&](int i, int s) -> int {
        const wg_range &r = ranges[i];
        return run(r.batch, p, action ? action + r.action_offset : nullptr, action_cols, action_stride, action_step,
                   r.outputs, 1, r.plan, r.plan_blocks, r.stream, true, false, false, s);
    };
    // A launch-time failure (hipGetLastError after a launch) can still stop the issue part-way, after other ranges or
    // steps went out: the call then returns that error with a partially stepped batch, but the side streams are joined
    // back to ranges[0].stream first, so the caller's stream never runs ahead of work the call did issue.
    int rc = 0;
    for (int s = 0; s < n_steps && !rc; s++)
        for (int i = 0; i < n && !rc; i++) rc = issue(i, s);
    for (int i = 1; i < n; i++)
        if (hipEventRecord(events[i], ranges[i].stream) != hipSuccess || hipStreamWaitEvent(s0, events[i], 0) != hipSuccess)
            return rc ? rc : fail(WG_EHIP, "join event failed");
    return rc;
}

int wg_step_ranges(const wg_range *ranges, int32_t n, const wg_params *p, const float *action, int32_t action_cols,
                   int32_t action_stride, hipEvent_t *events) {
    return wg_run_ranges(ranges, n, p, action, action_cols, action_stride, 0, 1, events);
}

int wg_observe(const wg_batch *b, const wg_params *p, const wg_outputs *o, const int32_t *plan,
               int32_t plan_blocks, hipStream_t stream) {
    if (!o) return fail(WG_EINVAL, "null outputs");
    return run(b, p, nullptr, 0, 0, 0, o, 1, plan, plan_blocks, stream, false);
}

// SURVEY §8(b)'s declared signatures (ABI 13): uniform batches only (a ragged batch needs a plan)
int wg_step_simple(const wg_batch *b, const float *action, const wg_params *p, int32_t n_steps, hipStream_t stream) {
    if (b && b->ragged) return fail(WG_EINVAL, "wg_step_simple: uniform batches only (ragged: wg_step with a plan)");
    const int32_t A = b ? b->A : 0;
    const int64_t step = b ? (int64_t)b->N * A : 0;
    return run(b, p, A > 0 ? action : nullptr, A, A, step, nullptr, n_steps, nullptr, 0, stream, true);
}

int wg_observe_simple(const wg_batch *b, const wg_obs_cfg *cfg, float *obs, float *reward, uint8_t *done,
                      float *centroid, float *energy, hipStream_t stream) {
    if (b && b->ragged) return fail(WG_EINVAL, "wg_observe_simple: uniform batches only (ragged: wg_observe with a plan)");
    if (!b || !cfg) return fail(WG_EINVAL, "null batch / cfg");
    wg_outputs o{};
    o.obs = obs;
    o.obs_stride = 3 * (cfg->in3d ? 3 : 2) * b->M + (cfg->conmid ? 3 : 0) + b->A;
    o.reward = reward;
    o.done = done;
    o.centroid = centroid;
    o.energy = energy;
    return run(b, cfg, nullptr, 0, 0, 0, &o, 1, nullptr, 0, stream, false);
}

// ABI 14, a measurement aid (bench.py's roofline): wg_step's n_steps, one launch per step, each step kernel launched with
// a start and an end event of its own (hipExtLaunchKernel: the dispatch's own timestamps, so the launch gaps of
// back-to-back launches are not counted); waits for the stream, then *ms_per_launch = the mean kernel duration.
int wg_time_step(const wg_batch *b, const wg_params *p, const float *action, int32_t action_cols, int32_t action_stride,
                 int64_t action_step, const wg_outputs *o, int32_t n_steps, const int32_t *plan, int32_t plan_blocks,
                 hipStream_t stream, float *ms_per_launch) {
    if (!ms_per_launch || n_steps < 1) return fail(WG_EINVAL, "wg_time_step: n_steps >= 1 and ms_per_launch required");
    int rc = run(b, p, action, action_cols, action_stride, action_step, o, n_steps, plan, plan_blocks, stream, true,
                 false, true);   // every argument checked before the first launch
    if (rc) return rc;
    if (b->N == 0) return fail(WG_EINVAL, "wg_time_step: empty batch (no launch to time)");
    std::vector<hipEvent_t> ev((size_t)2 * n_steps, nullptr);
    for (auto &e : ev)
        if (hipEventCreate(&e) != hipSuccess) { rc = fail(WG_EHIP, "wg_time_step: event create failed"); break; }
    for (int s = 0; s < n_steps && !rc; s++) {
        g_kev_start = ev[2 * s]; g_kev_stop = ev[2 * s + 1];
        rc = run(b, p, action, action_cols, action_stride, action_step, o, 1, plan, plan_blocks, stream, true, false,
                 false, s);
    }
    g_kev_start = g_kev_stop = nullptr;
    double total = 0.0;
    // (after a failure part-way, the launches already issued still hold their events: wait for them before destroying)
    if (hipStreamSynchronize(stream) != hipSuccess && !rc) rc = fail(WG_EHIP, "wg_time_step: stream sync failed");
    for (int s = 0; s < n_steps && !rc; s++) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, ev[2 * s], ev[2 * s + 1]) != hipSuccess)
            rc = fail(WG_EHIP, "wg_time_step: elapsed time of step %d unavailable", s);
        total += ms;
    }
    for (auto e : ev)
        if (e) (void)hipEventDestroy(e);
    if (!rc) *ms_per_launch = (float)(total / n_steps);
    return rc;
}

int wg_reset(const wg_batch *b, const wg_params *p, const float *noise, const uint8_t *mask, hipStream_t stream) {
    if (!p) return fail(WG_EINVAL, "null params");
    return reset_impl(b, noise, mask, p->in3d ? 1 : 0, stream);
}

int wg_reset_noise(const wg_batch *b, const float *noise, hipStream_t stream) {
    // every component except an exact +0.0: a 2D caller's z = +0.0 leaves v.z as it is (-0.0 included)
    return reset_impl(b, noise, nullptr, 2, stream);
}

int wg_wave_edge_passes(int32_t M, int32_t K) { return wave_passes(M, K); }

int wg_plan_errors(int32_t clear) {
    int v = 0;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_plan_error), sizeof v, 0, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(WG_EHIP, "plan error flag copy failed");
    if (clear && v) {
        const int z = 0;
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_plan_error), &z, sizeof z, 0, hipMemcpyHostToDevice) != hipSuccess)
            return fail(WG_EHIP, "plan error flag reset failed");
    }
    return v;
}

int wg_plan_waves(const int32_t *mass_off, const int32_t *edge_off, const int32_t *muscle_off, int32_t N,
                  int32_t *plan, int32_t max_tiles) {
    if (!mass_off || !edge_off || !muscle_off || !plan || N < 0 || max_tiles < 1)
        return fail(WG_EINVAL, "bad plan args");
    int Mmax = 1, Kmax = 0;
    for (int w = 0; w < N; w++) {
        Mmax = std::max(Mmax, mass_off[w + 1] - mass_off[w]);
        Kmax = std::max(Kmax, edge_off[w + 1] - edge_off[w]);
    }
    const int ne = wave_passes(Mmax, Kmax);
    if (!ne) return fail(WG_EINVAL, "a walker does not fit one wave (M=%d K=%d)", Mmax, Kmax);
    int tiles = 0, w = 0;
    plan[0] = 0;
    while (w < N) {
        int P = 0, E = 0, U = 0, n = 0;
        while (w < N) {
            const int m = mass_off[w + 1] - mass_off[w], k = edge_off[w + 1] - edge_off[w],
                      a = muscle_off[w + 1] - muscle_off[w];
            if (m > 64 || a > 64 || k > 64 * ne) return fail(WG_EINVAL, "walker %d does not fit one wave", w);
            if (n > 0 && (P + m > 64 || E + k > 64 * ne || U + a > 64 || n + 1 > RW_MAXW)) break;
            P += m; E += k; U += a; n++; w++;
        }
        if (tiles + 1 > max_tiles) return fail(WG_ERANGE, "plan needs more than %d tiles", max_tiles);
        plan[++tiles] = w;
    }
    return tiles;
}

int wg_plan_ragged(const int32_t *mass_off, const int32_t *edge_off, const int32_t *muscle_off,
                   int32_t N, int32_t *plan, int32_t max_blocks) {
    if (!mass_off || !edge_off || !muscle_off || !plan || N < 0 || max_blocks < 1)
        return fail(WG_EINVAL, "bad plan args");
    int blocks = 0;
    plan[0] = 0;
    int w = 0;
    while (w < N) {
        int P = 0, E = 0, U = 0, n = 0;
        while (w < N) {
            const int m = mass_off[w + 1] - mass_off[w], k = edge_off[w + 1] - edge_off[w],
                      a = muscle_off[w + 1] - muscle_off[w];
            if (n > 0 && (P + m > RAG_P || E + k > RAG_E || U + a > RAG_U || n + 1 > RAG_W)) break;
            P += m; E += k; U += a; n++; w++;
        }
        if (blocks + 1 > max_blocks) return fail(WG_ERANGE, "plan needs more than %d blocks", max_blocks);
        plan[++blocks] = w;
    }
    return blocks;
}

// the launch floor beside a small step (bench.py)
int wg_launch_floor(int32_t mode, int32_t blocks, int32_t threads, const float *in, float *out, int32_t n_launches,
                    hipStream_t stream) {
    if (blocks < 1 || threads < 1 || threads > 1024 || n_launches < 0 || mode < 0 || mode > 2 ||
        (mode >= 1 && (!in || !out)))
        return fail(WG_EINVAL, "bad floor launch (mode %d, %d x %d)", mode, blocks, threads);
    for (int i = 0; i < n_launches; i++) {
        if (mode == 0)
            hipLaunchKernelGGL(floor_empty_kernel, dim3(blocks), dim3(threads), 0, stream, out);
        else if (mode == 1)
            hipLaunchKernelGGL(floor_load_store_kernel, dim3(blocks), dim3(threads), 0, stream, in, out);
        else
            hipLaunchKernelGGL(floor_busy_kernel, dim3(blocks), dim3(threads), 0, stream, in, out);
    }
    return hipGetLastError() == hipSuccess ? 0 : fail(WG_EHIP, "floor launch failed");
}

// diagnostic builds (-DWG_STAMPS): copy n lean-wave stamp records (8 x u64 each) to host memory; WG_EINVAL otherwise
int wg_debug_stamps(unsigned long long *host, int n) {
#ifdef WG_STAMPS
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), (size_t)n * 8 * sizeof(unsigned long long), 0,
                            hipMemcpyDeviceToHost) != hipSuccess)
        return fail(WG_EHIP, "stamp copy failed");
    return 0;
#else
    (void)host; (void)n;
    return fail(WG_EINVAL, "not a stamps build");
#endif
}

int wg_launch_geometry(const wg_batch *b, wg_launch_info *info) {
    int rc = validate(b);
    if (rc) return rc;
    if (!info) return fail(WG_EINVAL, "null info");
    LeanGeo lg{};
    if (lean_geo(b, 0, &lg)) {   // the step kernel of uniform M | 64 batches
        info->threads = 64 * lg.wpb;
        info->walkers_per_block = lg.wpb * lg.wpw;
        info->blocks = lean_blocks(b, lg);
        info->lds_bytes = lg.wpb * lg.slice;
        return 0;
    }
    RagGeo rg{};
    if (b->ragged == 2 && lean_enabled() && rag_geo(b, 0, &rg)) {   // the wave kernel: one tile per wave
        info->threads = 64 * rg.wpb;
        info->walkers_per_block = -1;   // tiles hold whole walkers up to 64 masses: the plan decides
        info->blocks = -1;              // ceil(tiles / waves per workgroup), tiles from wg_plan_waves
        info->lds_bytes = rg.wpb * rg.slice;
        return 0;
    }
    const Geo g = b->ragged ? ragged_geo(b) : uniform_geo(b, 0);
    info->threads = g.threads;
    info->walkers_per_block = g.W;
    info->blocks = b->ragged ? -1 : (b->N + g.W - 1) / g.W;
    info->lds_bytes = g.lds;
    return 0;
}

}  // extern "C"
