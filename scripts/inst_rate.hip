// VALU issue cost per instruction kind (diagnostic, not product): each kernel runs one instruction kind as 8
// independent chains per lane (inline asm, so the instruction is exactly the one named), 8 waves per SIMD on every
// CU.  Prints one JSON line: per kind, the SIMD cycles one wave64 instruction occupies, relative to v_fma_f32 = 4
// (the clock-free figure: v_fma_f32 issues one wave64 instruction per 4 cycles on a 16-lane SIMD), and the clock
// that v_fma_f32's time implies.  Feeds the weighted cycle count of the canonical kernel.
// build: hipcc --offload-arch=gfx950 -O3 -o build_ablate/inst_rate scripts/inst_rate.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int ITERS = 2048, CH = 8;

// 32-bit register chains: x_c = op(x_c, y)
#define K32(name, INS)                                                                              \
    __global__ __launch_bounds__(256) void name(uint32_t *out, uint32_t y) {                          \
        uint32_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,     \
                 x6 = x0 + 6, x7 = x0 + 7;                                                            \
        for (int i = 0; i < ITERS; i++) {                                                              \
            asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS         \
                         " %3, %3, %8\n\t" INS " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" \
                         INS " %7, %7, %8"                                                             \
                         : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) \
                         : "v"(y));                                                                    \
        }                                                                                              \
        const uint32_t s = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;                                      \
        if (s == 0x12345678u) out[threadIdx.x] = s;                                                    \
    }
// 32-bit unary chains: x_c = op(x_c)
#define U32(name, INS)                                                                              \
    __global__ __launch_bounds__(256) void name(uint32_t *out, uint32_t y) {                          \
        uint32_t x0 = threadIdx.x + y, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5, \
                 x6 = x0 + 6, x7 = x0 + 7;                                                            \
        for (int i = 0; i < ITERS; i++) {                                                              \
            asm volatile(INS " %0, %0\n\t" INS " %1, %1\n\t" INS " %2, %2\n\t" INS " %3, %3\n\t" INS    \
                         " %4, %4\n\t" INS " %5, %5\n\t" INS " %6, %6\n\t" INS " %7, %7"                \
                         : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)); \
        }                                                                                              \
        const uint32_t s = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;                                      \
        if (s == 0x12345678u) out[threadIdx.x] = s;                                                    \
    }
// 64-bit register chains: x_c = op(x_c, y) (y a 64-bit register pair)
#define K64(name, INS)                                                                              \
    __global__ __launch_bounds__(256) void name(uint32_t *out, uint32_t yy) {                         \
        double y = (double)yy;                                                                         \
        double x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,       \
               x6 = x0 + 6, x7 = x0 + 7;                                                              \
        for (int i = 0; i < ITERS; i++) {                                                              \
            asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS         \
                         " %3, %3, %8\n\t" INS " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" \
                         INS " %7, %7, %8"                                                             \
                         : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) \
                         : "v"(y));                                                                    \
        }                                                                                              \
        const double s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;                                        \
        if (s == 12345.678) out[threadIdx.x] = 1;                                                      \
    }
// 64-bit unary chains: x_c = op(x_c)
#define U64(name, INS)                                                                              \
    __global__ __launch_bounds__(256) void name(uint32_t *out, uint32_t yy) {                         \
        double x0 = threadIdx.x + yy, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,  \
               x6 = x0 + 6, x7 = x0 + 7;                                                              \
        for (int i = 0; i < ITERS; i++) {                                                              \
            asm volatile(INS " %0, %0\n\t" INS " %1, %1\n\t" INS " %2, %2\n\t" INS " %3, %3\n\t" INS    \
                         " %4, %4\n\t" INS " %5, %5\n\t" INS " %6, %6\n\t" INS " %7, %7"                \
                         : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)); \
        }                                                                                              \
        const double s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;                                        \
        if (s == 12345.678) out[threadIdx.x] = 1;                                                      \
    }
// conversions between a 32-bit and a 64-bit register, in pairs (f32 -> f64 -> f32): the cost reported is per
// instruction, the mean of the two
#define CVT2(name, A, B)                                                                            \
    __global__ __launch_bounds__(256) void name(uint32_t *out, uint32_t yy) {                         \
        float x0 = threadIdx.x + yy, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;                            \
        double d0, d1, d2, d3;                                                                         \
        for (int i = 0; i < ITERS; i++) {                                                              \
            asm volatile(A " %4, %0\n\t" A " %5, %1\n\t" A " %6, %2\n\t" A " %7, %3\n\t" B " %0, %4\n\t" \
                         B " %1, %5\n\t" B " %2, %6\n\t" B " %3, %7"                                     \
                         : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3)); \
        }                                                                                              \
        const float s = x0 + x1 + x2 + x3;                                                             \
        if (s == 12345.678f) out[threadIdx.x] = 1;                                                     \
    }
// v_pk_fma_f32 / v_fma_f32 / v_fma_f64 in the three-operand form
#define F3(name, T, INS)                                                                            \
    __global__ __launch_bounds__(256) void name(uint32_t *out, uint32_t yy) {                         \
        T y = (T)yy;                                                                                   \
        T x0 = (T)threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,         \
          x6 = x0 + 6, x7 = x0 + 7;                                                                    \
        for (int i = 0; i < ITERS; i++) {                                                              \
            asm volatile(INS " %0, %0, %8, %8\n\t" INS " %1, %1, %8, %8\n\t" INS " %2, %2, %8, %8\n\t"  \
                         INS " %3, %3, %8, %8\n\t" INS " %4, %4, %8, %8\n\t" INS " %5, %5, %8, %8\n\t"  \
                         INS " %6, %6, %8, %8\n\t" INS " %7, %7, %8, %8"                                \
                         : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7) \
                         : "v"(y));                                                                    \
        }                                                                                              \
        const T s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;                                             \
        if (s == (T)12345.678) out[threadIdx.x] = 1;                                                   \
    }

F3(k_fma_f32, float, "v_fma_f32")
F3(k_fma_f64, double, "v_fma_f64")
typedef float f2 __attribute__((ext_vector_type(2)));
F3(k_pk_fma_f32, double, "v_pk_fma_f32")   // a 64-bit register pair holds the two floats
K32(k_add_u32, "v_add_u32")
K32(k_mul_u32_u24, "v_mul_u32_u24")
K32(k_mul_lo_u32, "v_mul_lo_u32")
K32(k_mul_f32, "v_mul_f32")
K32(k_xor_b32, "v_xor_b32")
K64(k_mul_f64, "v_mul_f64")
K64(k_add_f64, "v_add_f64")
U32(k_rcp_f32, "v_rcp_f32")
U32(k_sqrt_f32, "v_sqrt_f32")
U64(k_rcp_f64, "v_rcp_f64")
U64(k_sqrt_f64, "v_sqrt_f64")
CVT2(k_cvt, "v_cvt_f64_f32", "v_cvt_f32_f64")

// dependent chains (one chain per lane): launched with one wave per SIMD they give the issue-to-issue latency of a
// dependent instruction; with W waves per SIMD, how far W waves interleaving one chain each get towards the issue rate
__global__ __launch_bounds__(256) void d_fma_f32(uint32_t *out, uint32_t yy) {
    float x = threadIdx.x, y = (float)yy;
    for (int i = 0; i < ITERS; i++)
        asm volatile("v_fma_f32 %0, %0, %1, %1\n\tv_fma_f32 %0, %0, %1, %1\n\tv_fma_f32 %0, %0, %1, %1\n\t"
                     "v_fma_f32 %0, %0, %1, %1\n\tv_fma_f32 %0, %0, %1, %1\n\tv_fma_f32 %0, %0, %1, %1\n\t"
                     "v_fma_f32 %0, %0, %1, %1\n\tv_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(y));
    if (x == 12345.678f) out[threadIdx.x] = 1;
}
__global__ __launch_bounds__(256) void d_fma_f64(uint32_t *out, uint32_t yy) {
    double x = threadIdx.x, y = (double)yy;
    for (int i = 0; i < ITERS; i++)
        asm volatile("v_fma_f64 %0, %0, %1, %1\n\tv_fma_f64 %0, %0, %1, %1\n\tv_fma_f64 %0, %0, %1, %1\n\t"
                     "v_fma_f64 %0, %0, %1, %1\n\tv_fma_f64 %0, %0, %1, %1\n\tv_fma_f64 %0, %0, %1, %1\n\t"
                     "v_fma_f64 %0, %0, %1, %1\n\tv_fma_f64 %0, %0, %1, %1" : "+v"(x) : "v"(y));
    if (x == 12345.678) out[threadIdx.x] = 1;
}
// the mass loop's accumulation step a = f32(f64(a) + q) followed by the damping add, as one dependent chain of 4
__global__ __launch_bounds__(256) void d_acc(uint32_t *out, uint32_t yy) {
    float a = threadIdx.x, g = (float)yy;
    double q = (double)yy, t;
    for (int i = 0; i < ITERS; i++)
        asm volatile("v_cvt_f64_f32 %1, %0\n\tv_add_f64 %1, %1, %2\n\tv_cvt_f32_f64 %0, %1\n\tv_add_f32 %0, %0, %3\n\t"
                     "v_cvt_f64_f32 %1, %0\n\tv_add_f64 %1, %1, %2\n\tv_cvt_f32_f64 %0, %1\n\tv_add_f32 %0, %0, %3"
                     : "+v"(a), "=&v"(t) : "v"(q), "v"(g));
    if (a == 12345.678f) out[threadIdx.x] = 1;
}
// DPP row_shr:1 add chain (the per-walker sequential sums)
__global__ __launch_bounds__(256) void d_dpp(uint32_t *out, uint32_t yy) {
    float x = threadIdx.x, y = (float)yy;
    for (int i = 0; i < ITERS; i++)
        asm volatile("v_add_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                     "v_add_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                     "v_add_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                     "v_add_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                     "v_add_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                     "v_add_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                     "v_add_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                     "v_add_f32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(x) : "v"(y));
    if (x == 12345.678f) out[threadIdx.x] = 1;
}
// ds_bpermute throughput: 8 independent gathers per iteration (the spring phase's endpoint gathers)
__global__ __launch_bounds__(256) void k_bperm(uint32_t *out, uint32_t yy) {
    int a = (threadIdx.x ^ yy) << 2, v0 = threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5,
        v6 = v0 + 6, v7 = v0 + 7;
    for (int i = 0; i < ITERS; i++) {
        v0 = __builtin_amdgcn_ds_bpermute(a, v0); v1 = __builtin_amdgcn_ds_bpermute(a, v1);
        v2 = __builtin_amdgcn_ds_bpermute(a, v2); v3 = __builtin_amdgcn_ds_bpermute(a, v3);
        v4 = __builtin_amdgcn_ds_bpermute(a, v4); v5 = __builtin_amdgcn_ds_bpermute(a, v5);
        v6 = __builtin_amdgcn_ds_bpermute(a, v6); v7 = __builtin_amdgcn_ds_bpermute(a, v7);
    }
    if ((v0 ^ v1 ^ v2 ^ v3 ^ v4 ^ v5 ^ v6 ^ v7) == 0x12345678) out[threadIdx.x] = 1;
}

typedef void (*kfn)(uint32_t *, uint32_t);
struct Kind { const char *name; kfn k; double per_iter; };   // per_iter: instructions per chain iteration

int main() {
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    const int blocks = pr.multiProcessorCount * 8;   // 8 workgroups of 4 waves per CU: 8 waves per SIMD
    uint32_t *d;
    CK(hipMalloc(&d, 256 * sizeof(uint32_t)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const Kind kinds[] = {
        {"v_fma_f32", k_fma_f32, 8}, {"v_pk_fma_f32", k_pk_fma_f32, 8}, {"v_fma_f64", k_fma_f64, 8},
        {"v_mul_f64", k_mul_f64, 8}, {"v_add_f64", k_add_f64, 8}, {"v_mul_f32", k_mul_f32, 8},
        {"v_add_u32", k_add_u32, 8}, {"v_xor_b32", k_xor_b32, 8}, {"v_mul_u32_u24", k_mul_u32_u24, 8},
        {"v_mul_lo_u32", k_mul_lo_u32, 8}, {"v_rcp_f32", k_rcp_f32, 8}, {"v_sqrt_f32", k_sqrt_f32, 8},
        {"v_rcp_f64", k_rcp_f64, 8}, {"v_sqrt_f64", k_sqrt_f64, 8}, {"v_cvt_f64_f32+v_cvt_f32_f64", k_cvt, 8},
    };
    const int nk = sizeof(kinds) / sizeof(kinds[0]);
    double ms_per_inst[32];
    for (int v = 0; v < nk; v++) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; rep++) {
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(kinds[v].k, dim3(blocks), dim3(256), 0, 0, d, 3u);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep > 0 && ms < best) best = ms;
        }
        ms_per_inst[v] = best / (ITERS * kinds[v].per_iter);
    }
    // waves per SIMD = 8, so one SIMD issues 8 * ITERS * per_iter wave-instructions; v_fma_f32 = 4 cycles each
    const double ref = ms_per_inst[0];
    const double waves_per_simd = 8.0;
    const double clk_ghz = 4.0 * waves_per_simd / (ref * 1e-3) / 1e9;
    printf("{\"cus\": %d, \"clock_ghz_implied\": %.3f, \"cycles_per_wave_instruction\": {", pr.multiProcessorCount,
           clk_ghz);
    for (int v = 0; v < nk; v++)
        printf("%s\"%s\": %.2f", v ? ", " : "", kinds[v].name, 4.0 * ms_per_inst[v] / ref);
    printf("}");
    // dependent chains at W waves per SIMD (W workgroups of 4 waves per CU): SIMD cycles per chain instruction per
    // wave, at the clock implied above (cycles between two dependent instructions of one wave when W = 1)
    const Kind deps[] = {{"dep v_fma_f32", d_fma_f32, 8}, {"dep v_fma_f64", d_fma_f64, 8},
                         {"dep cvt+add_f64+cvt+add_f32 (per instruction)", d_acc, 8},
                         {"dep v_add_f32_dpp row_shr", d_dpp, 8}, {"ds_bpermute_b32 (8 independent)", k_bperm, 8}};
    printf(", \"dependent_chain_cycles_per_instruction\": {");
    for (int v = 0; v < (int)(sizeof(deps) / sizeof(deps[0])); v++) {
        printf("%s\"%s\": {", v ? ", " : "", deps[v].name);
        const int ws[] = {1, 2, 4, 6, 8};
        for (int wi = 0; wi < 5; wi++) {
            float best = 1e30f;
            for (int rep = 0; rep < 4; rep++) {
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(deps[v].k, dim3(pr.multiProcessorCount * ws[wi]), dim3(256), 0, 0, d, 3u);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep > 0 && ms < best) best = ms;
            }
            // one SIMD runs ws waves, each ITERS * per_iter instructions in its chain: cycles per (wave, instruction)
            const double cyc = best * 1e-3 * clk_ghz * 1e9 / (ITERS * deps[v].per_iter);
            printf("%s\"w%d\": %.2f", wi ? ", " : "", ws[wi], cyc / ws[wi]);
        }
        printf("}");
    }
    printf("}}\n");
    return 0;
}
