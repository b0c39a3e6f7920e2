// Exhaustive GPU check: rcp64_nr(m) (v_rcp_f64 + two Newton steps, walker_hip.hip) equals the IEEE RN64(1/m) for every
// float32 m with |m| in [2^-20, 2^21) (the divisor range the kernels' fast quotients require; divisor_ok), both signs.
// Markstein: a Newton step y + y(1 - m y) (two FMAs) from a y within one ulp of 1/m is correctly rounded unless m's
// 53-bit significand is all ones, which a float32 m cannot have; this checks it on the hardware, every input.
// build: hipcc --offload-arch=gfx950 -O3 -o build_ablate/check_rcp64 scripts/check_rcp64.hip ; run on the GPU box.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ double rcp64_nr(double d) {   // (as walker_hip.hip)
    double y = __builtin_amdgcn_rcp(d);
    double e = __builtin_fma(-d, y, 1.0);
    y = __builtin_fma(y, e, y);
    e = __builtin_fma(-d, y, 1.0);
    return __builtin_fma(y, e, y);
}

__global__ void check(uint32_t lo, uint32_t n, unsigned long long *bad, uint32_t *first) {
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        const uint32_t bits = lo + k;
        for (int s = 0; s < 2; s++) {
            const float m = __uint_as_float(bits | (s ? 0x80000000u : 0u));
            const double d = (double)m;
            const double a = rcp64_nr(d), b = 1.0 / d;
            if (__double_as_longlong(a) != __double_as_longlong(b)) {
                atomicAdd(bad, 1ull);
                atomicMin(first, bits);
            }
        }
    }
}

int main() {
    const uint32_t lo = 0x35800000u;   // 2^-20
    const uint32_t hi = 0x4a000000u;   // 2^21
    unsigned long long *bad; uint32_t *first;
    hipMalloc(&bad, sizeof *bad); hipMalloc(&first, sizeof *first);
    hipMemset(bad, 0, sizeof *bad); hipMemset(first, 0xff, sizeof *first);
    hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, lo, hi - lo, bad, first);
    unsigned long long h = 0; uint32_t f = 0;
    hipMemcpy(&h, bad, sizeof h, hipMemcpyDeviceToHost); hipMemcpy(&f, first, sizeof f, hipMemcpyDeviceToHost);
    printf("{\"check\": \"rcp64_nr(m) == RN64(1/m)\", \"range\": \"|m| in [2^-20, 2^21), both signs\", "
           "\"inputs\": %llu, \"mismatches\": %llu, \"first_bad_bits\": \"0x%08x\"}\n",
           2ull * (unsigned long long)(hi - lo), h, h ? f : 0u);
    return h != 0;
}
