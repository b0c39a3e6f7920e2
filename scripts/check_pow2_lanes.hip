// Exhaustive GPU check (profiling / verification aid, not product): pw_pow2_lanes (walker_hip.hip: glibc's powf tables
// held in lane registers and read by ds_bpermute) and pw_pow2_lds (the tables in LDS) give the bits of pw_pow2 (powf2.h, itself pinned exhaustively
// against libm by scripts/check_powf2.c) for every float32 bit pattern with the sign clear (zero, subnormals, normals,
// inf, NaNs), and for the same patterns with the sign set.  Built against the product source itself.
// build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I include -o ab_session/check_pow2_lanes
//        scripts/check_pow2_lanes.hip ; run on the GPU box.
#include "../walker_gym_amd/csrc/walker_hip.hip"

__global__ void check_pow2_lanes(unsigned long long *bad, uint32_t *first) {
    const int lane = threadIdx.x & 63;
    const double tl = PW_LOG2_TAB[lane & 31], te = pw_asdouble(PW_EXP2_TAB[lane & 31]);
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    // wave-uniform trip counts: every lane of a wave takes part in each gather
    for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~63u); base < (1ull << 32); base += stride) {
        const uint32_t bits = (uint32_t)(base + lane);
        const float x = __uint_as_float(bits);
        const float a = pw_pow2(x), b = pw_pow2_lanes(x, tl, te);
        if (__float_as_uint(a) != __float_as_uint(b) && !(a != a && b != b)) {
            atomicAdd(bad, 1ull);
            atomicMin(first, bits);
        }
    }
}

__global__ void check_pow2_lds(unsigned long long *bad, uint32_t *first) {
    pw_tables_to_lds(threadIdx.x);
    __syncthreads();
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < (1ull << 32); k += stride) {
        const uint32_t bits = (uint32_t)k;
        const float x = __uint_as_float(bits);
        const float a = pw_pow2(x), b = pw_pow2_lds(x);
        if (__float_as_uint(a) != __float_as_uint(b) && !(a != a && b != b)) {
            atomicAdd(bad, 1ull);
            atomicMin(first, bits);
        }
    }
}

// pw_pow2_fast's claim on the device (its band from v_frexp_exp / v_ldexp): RN(x*x) only where pw_pow2 agrees
__global__ void check_pow2_fast(unsigned long long *bad, uint32_t *first) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < (1ull << 32); k += stride) {
        const uint32_t bits = (uint32_t)k;
        const float x = __uint_as_float(bits);
        float f;
        if ((bits & 0x7fffffffu) < 0x7f800000u && pw_pow2_fast(x, &f) && __float_as_uint(f) != __float_as_uint(pw_pow2(x))) {
            atomicAdd(bad, 1ull);
            atomicMin(first, bits);
        }
    }
}

int main() {
    unsigned long long *bad; uint32_t *first;
    hipMalloc(&bad, sizeof *bad); hipMalloc(&first, sizeof *first);
    hipMemset(bad, 0, sizeof *bad); hipMemset(first, 0xff, sizeof *first);
    hipLaunchKernelGGL(check_pow2_lanes, dim3(8192), dim3(256), 0, 0, bad, first);
    unsigned long long h = 0; uint32_t f = 0;
    hipMemcpy(&h, bad, sizeof h, hipMemcpyDeviceToHost); hipMemcpy(&f, first, sizeof f, hipMemcpyDeviceToHost);
    printf("{\"check\": \"pw_pow2_lanes(x) == pw_pow2(x)\", \"range\": \"every float32 bit pattern\", "
           "\"inputs\": %llu, \"mismatches\": %llu, \"first_bad_bits\": \"0x%08x\"}\n", 1ull << 32, h, h ? f : 0u);
    unsigned long long h2 = 0; uint32_t f2 = 0;
    hipMemset(bad, 0, sizeof *bad); hipMemset(first, 0xff, sizeof *first);
    hipLaunchKernelGGL(check_pow2_lds, dim3(8192), dim3(256), 0, 0, bad, first);
    hipMemcpy(&h2, bad, sizeof h2, hipMemcpyDeviceToHost); hipMemcpy(&f2, first, sizeof f2, hipMemcpyDeviceToHost);
    printf("{\"check\": \"pw_pow2_lds(x) == pw_pow2(x)\", \"range\": \"every float32 bit pattern\", "
           "\"inputs\": %llu, \"mismatches\": %llu, \"first_bad_bits\": \"0x%08x\"}\n", 1ull << 32, h2, h2 ? f2 : 0u);
    unsigned long long h3 = 0; uint32_t f3 = 0;
    hipMemset(bad, 0, sizeof *bad); hipMemset(first, 0xff, sizeof *first);
    hipLaunchKernelGGL(check_pow2_fast, dim3(8192), dim3(256), 0, 0, bad, first);
    hipMemcpy(&h3, bad, sizeof h3, hipMemcpyDeviceToHost); hipMemcpy(&f3, first, sizeof f3, hipMemcpyDeviceToHost);
    printf("{\"check\": \"pw_pow2_fast(x) claims only pw_pow2(x)\", \"range\": \"every finite float32\", "
           "\"inputs\": %llu, \"mismatches\": %llu, \"first_bad_bits\": \"0x%08x\"}\n", 1ull << 32, h3, h3 ? f3 : 0u);
    return h != 0 || h2 != 0 || h3 != 0;
}
