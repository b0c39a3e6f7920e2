// VALU peak microbenchmark (diagnostic, not product): the FP64 and FP32 vector FLOP/s one MI355X sustains, the
// denominators of bench.py's pair-force rooflines.  Each lane runs 8 independent FMA chains (enough to cover the
// dependent-issue latency), 8 waves per SIMD, 8 x 256 CUs of workgroups; FLOP = 2 per FMA per lane.
//   f64      v_fma_f64
//   f32      v_fma_f32 (one lane-FLOP pair per instruction: the non-packed rate)
//   f32_pk   v_pk_fma_f32 (two per instruction: the 157.3 TFLOP/s spec rate)
// build: hipcc --offload-arch=gfx950 -O3 -o build_ablate/valu_peak scripts/valu_peak.hip
// prints one JSON line: TFLOP/s per variant and the clock-independent ratio f64 / f32_pk.
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096, CH = 8;

__global__ __launch_bounds__(256) void k_f64(double *out, double a, double b) {
    double x[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) x[c] = __builtin_fma(x[c], a, b);
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s += x[c];
    if (s == 12345.678) out[threadIdx.x] = s;   // never true: keeps the chains live
}

__global__ __launch_bounds__(256) void k_f32(float *out, float a, float b) {
    float x[CH];
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = threadIdx.x * 1e-3f + c;
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) x[c] = __builtin_fmaf(x[c], a, b);
        asm volatile("" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s += x[c];
    if (s == 12345.678f) out[threadIdx.x] = s;
}

typedef float f2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_f32pk(float *out, float a, float b) {
    f2 x[CH];
    const f2 av = {a, a}, bv = {b, b};
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = f2{threadIdx.x * 1e-3f + c, c * 0.5f};
    for (int i = 0; i < ITERS; i++) {
#pragma unroll
        for (int c = 0; c < CH; c++) x[c] = __builtin_elementwise_fma(x[c], av, bv);
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < CH; c++) s += x[c].x + x[c].y;
    if (s == 12345.678f) out[threadIdx.x] = s;
}

int main() {
    int dev = 0;
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, dev));
    const int blocks = pr.multiProcessorCount * 8;   // 8 workgroups of 4 waves per CU: 8 waves per SIMD
    double *d64;
    float *d32;
    CK(hipMalloc(&d64, 256 * sizeof(double)));
    CK(hipMalloc(&d32, 256 * sizeof(float)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double lanes = (double)blocks * 256;
    double tf[3];
    for (int v = 0; v < 3; v++) {
        float best = 1e30f;
        for (int rep = 0; rep < 5; rep++) {
            CK(hipEventRecord(e0));
            if (v == 0) hipLaunchKernelGGL(k_f64, dim3(blocks), dim3(256), 0, 0, d64, 0.999999, 1e-7);
            else if (v == 1) hipLaunchKernelGGL(k_f32, dim3(blocks), dim3(256), 0, 0, d32, 0.999999f, 1e-7f);
            else hipLaunchKernelGGL(k_f32pk, dim3(blocks), dim3(256), 0, 0, d32, 0.999999f, 1e-7f);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep > 0 && ms < best) best = ms;
        }
        const double flop = lanes * ITERS * CH * 2.0 * (v == 2 ? 2.0 : 1.0);
        tf[v] = flop / (best * 1e-3) / 1e12;
    }
    printf("{\"cus\": %d, \"f64_fma_tflops\": %.2f, \"f32_fma_tflops\": %.2f, \"f32_pk_fma_tflops\": %.2f, "
           "\"f64_over_f32pk\": %.3f}\n", pr.multiProcessorCount, tf[0], tf[1], tf[2], tf[0] / tf[2]);
    return 0;
}
