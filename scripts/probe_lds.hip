// LDS throughput probe (diagnostic, not product): chip-wide time of N independent LDS operations per lane for
// ds_bpermute_b32, ds_read_b32 (random / linear), ds_read_b64, ds_read_b128 and ds_write_b32 at a given number of
// waves per CU.  Build: hipcc --offload-arch=gfx950 -O3 -o scripts/probe_lds scripts/probe_lds.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int ITERS = 2048;

template <int OP>
__global__ __launch_bounds__(256) void probe(float *out, int seed) {
    __shared__ __attribute__((aligned(16))) float lds[256 * 16];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 256 * 16; i += 256) lds[i] = (float)(i ^ seed);
    __syncthreads();
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
    unsigned r = (unsigned)(lane * 2654435761u) ^ (unsigned)seed;
    const int wbase = (tid >> 6) * 1024;   // this wave's 4 KB slice (floats)
    for (int it = 0; it < ITERS; it++) {
        r = r * 1664525u + 1013904223u;
        const int a0 = (r >> 8) & 1023, a1 = (r >> 12) & 1023, a2 = (r >> 16) & 1023, a3 = (r >> 20) & 1023;
        if (OP == 0) {   // bpermute, random source lanes
            acc0 += __int_as_float(__builtin_amdgcn_ds_bpermute((a0 & 63) << 2, (int)r + 0));
            acc1 += __int_as_float(__builtin_amdgcn_ds_bpermute((a1 & 63) << 2, (int)r + 1));
            acc2 += __int_as_float(__builtin_amdgcn_ds_bpermute((a2 & 63) << 2, (int)r + 2));
            acc3 += __int_as_float(__builtin_amdgcn_ds_bpermute((a3 & 63) << 2, (int)r + 3));
        } else if (OP == 1) {   // ds_read_b32 random within the slice
            acc0 += lds[wbase + a0]; acc1 += lds[wbase + a1]; acc2 += lds[wbase + a2]; acc3 += lds[wbase + a3];
        } else if (OP == 2) {   // ds_read_b32 linear (conflict-free)
            const int o = (it * 4) & 1023;
            acc0 += lds[wbase + ((o + lane) & 1023)]; acc1 += lds[wbase + ((o + 64 + lane) & 1023)];
            acc2 += lds[wbase + ((o + 128 + lane) & 1023)]; acc3 += lds[wbase + ((o + 192 + lane) & 1023)];
        } else if (OP == 3) {   // ds_read_b64 random (8-B aligned)
            const float2 *l2 = reinterpret_cast<const float2 *>(lds + wbase);
            const float2 x = l2[a0 & 511], y = l2[a1 & 511];
            acc0 += x.x; acc1 += x.y; acc2 += y.x; acc3 += y.y;
        } else if (OP == 4) {   // ds_read_b128 random (16-B aligned)
            const float4 *l4 = reinterpret_cast<const float4 *>(lds + wbase);
            const float4 x = l4[a0 & 255];
            acc0 += x.x; acc1 += x.y; acc2 += x.z; acc3 += x.w;
        } else if (OP == 5) {   // ds_write_b32 linear
            const int o = (it * 4) & 1023;
            lds[wbase + ((o + lane) & 1023)] = acc0 + it; lds[wbase + ((o + 64 + lane) & 1023)] = acc1 + it;
            acc0 += 1.f; acc1 += 2.f;
        } else if (OP == 6) {   // ds_read_b64 random pair at 24-B record stride (the spring-term reads)
            const double *ld = reinterpret_cast<const double *>(lds + wbase);
            const int e = a0 % 160;
            acc0 += (float)ld[3 * e]; acc1 += (float)ld[3 * e + 1]; acc2 += (float)ld[3 * e + 2];
        }
    }
    out[blockIdx.x * 256 + tid] = acc0 + acc1 + acc2 + acc3;
}

template <int OP>
float run(int blocks, float *d) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    probe<OP><<<blocks, 256>>>(d, 1);
    hipEventRecord(e0);
    for (int k = 0; k < 5; k++) probe<OP><<<blocks, 256>>>(d, k);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main(int argc, char **argv) {
    const int per_cu = argc > 1 ? atoi(argv[1]) : 4;   // workgroups (of 4 waves) per CU
    const int blocks = 256 * per_cu;
    float *d;
    hipMalloc(&d, (size_t)blocks * 256 * 4);
    const char *names[] = {"bpermute", "read_b32_rand", "read_b32_lin", "read_b64_rand", "read_b128_rand", "write_b32_lin",
                           "read_b64_rec24"};
    const int ops_per_it[] = {4, 4, 4, 2, 1, 2, 3};
    float ms[7];
    ms[0] = run<0>(blocks, d); ms[1] = run<1>(blocks, d); ms[2] = run<2>(blocks, d); ms[3] = run<3>(blocks, d);
    ms[4] = run<4>(blocks, d); ms[5] = run<5>(blocks, d); ms[6] = run<6>(blocks, d);
    for (int i = 0; i < 7; i++) {
        const double insts_per_cu = (double)per_cu * 4 * ITERS * ops_per_it[i];
        printf("{\"op\": \"%s\", \"waves_per_cu\": %d, \"ms\": %.4f, \"ns_per_wave_inst_per_cu\": %.3f}\n", names[i],
               per_cu * 4, ms[i], ms[i] * 1e6 / insts_per_cu);
    }
    hipFree(d);
    return 0;
}
