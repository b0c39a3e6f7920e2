// Memory-skeleton experiment (diagnostic, not product): how fast can the step kernel's HBM traffic
// move with NO physics?  Canonical batch (N=65536, M=16, K=40, A=8, obs 152 floats), W=16 walkers
// per 256-thread workgroup, the product's array layout.  Variants:
//   copy   : one flat float4 stream of the same total read / write bytes (achievable bandwidth)
//   skel   : per-workgroup reads of every input span + writes of every output span, loads issued
//            up front, no compute (the product kernel's access pattern)
//   skel_nt: skel with nontemporal stores
// build: hipcc --offload-arch=gfx950 -O3 -o build_ablate/membench scripts/membench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int N = 65536, M = 16, K = 40, A = 8, D = 152, W = 16, T = 256;

struct Bufs {
    float *pos, *vel, *acc, *mass, *mx, *bounds, *action, *obs, *reward, *energy, *centroid;
    uint4 *edges;
    uint32_t *inc;
    uint16_t *inc_off;
    int *steps;
    uint8_t *contact, *done;
};

typedef float vf4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ inline void st4(float4 *p, float4 v) {
    vf4 x = {v.x, v.y, v.z, v.w};
    if (NT) __builtin_nontemporal_store(x, reinterpret_cast<vf4 *>(p));
    else *reinterpret_cast<vf4 *>(p) = x;
}

template <bool NT>
__global__ __launch_bounds__(256) void skel(Bufs b) {
    __shared__ float4 tile[1024];
    const int tid = threadIdx.x, w0 = blockIdx.x * W;
    const size_t P0 = (size_t)w0 * M, E0 = (size_t)w0 * K, U0 = (size_t)w0 * A;
    const int n3 = 3 * W * M / 4;                        // 192 float4 of pos (and of vel)
    float4 pp = reinterpret_cast<const float4 *>(b.pos + 3 * P0)[min(tid, n3 - 1)];
    float4 pv = reinterpret_cast<const float4 *>(b.vel + 3 * P0)[min(tid, n3 - 1)];
    uint4 pi = reinterpret_cast<const uint4 *>(b.inc + E0 / 1)[min(tid, W * K / 4 - 1)];   // 2 u16 per edge
    uint4 e0 = b.edges[E0 + tid], e1 = b.edges[E0 + tid + T], e2 = b.edges[E0 + min(tid + 2 * T, W * K - 1)];
    float m = b.mass[P0 + tid];
    float mx = b.mx[U0 + (tid & 127)];
    float2 bd = reinterpret_cast<const float2 *>(b.bounds)[U0 + (tid & 127)];
    float ac = b.action[U0 + (tid & 127)];
    uint16_t io = b.inc_off[P0 + w0 + min(tid, W * (M + 1) - 1)];
    int st = b.steps[w0 + (tid & 15)];
    // fold everything into the LDS tile so nothing is dead
    float s = pp.x + pv.y + m + mx + bd.x + ac + (float)io + (float)st + __uint_as_float(pi.x ^ e0.y ^ e1.z ^ e2.w);
    tile[tid] = make_float4(s, pp.y, pv.x, pp.z);
    __syncthreads();
    // writes: pos, vel, acc (3 x 192 float4), obs (W*D/4 = 608 float4), per-walker outputs
    if (tid < n3) {
        st4<NT>(reinterpret_cast<float4 *>(b.pos + 3 * P0) + tid, tile[tid]);
        st4<NT>(reinterpret_cast<float4 *>(b.vel + 3 * P0) + tid, tile[(tid + 1) & 255]);
        st4<NT>(reinterpret_cast<float4 *>(b.acc + 3 * P0) + tid, tile[(tid + 2) & 255]);
    }
    float4 *ob = reinterpret_cast<float4 *>(b.obs + (size_t)w0 * D);
    for (int i = tid; i < W * D / 4; i += T) st4<NT>(ob + i, tile[i & 255]);
    if (tid < W * A) b.mx[U0 + tid] = tile[tid].x;
    b.contact[P0 + tid] = (uint8_t)tid;
    if (tid < W) {
        b.steps[w0 + tid] = st + 1;
        b.reward[w0 + tid] = s; b.energy[w0 + tid] = s; b.done[w0 + tid] = 0;
        b.centroid[3 * (w0 + tid)] = s; b.centroid[3 * (w0 + tid) + 1] = s; b.centroid[3 * (w0 + tid) + 2] = s;
    }
}

__global__ void copy(const float4 *__restrict__ src, float4 *__restrict__ dst, size_t nr, size_t nw) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
    float4 acc = make_float4(0, 0, 0, 0);
    for (size_t k = i; k < nr; k += stride) { float4 v = src[k]; acc.x += v.x; acc.y += v.y; }
    for (size_t k = i; k < nw; k += stride) dst[k] = make_float4(acc.x, acc.y, (float)k, 0.f);
}

int main() {
    const size_t P = (size_t)N * M, E = (size_t)N * K, U = (size_t)N * A;
    Bufs b{};
    CK(hipMalloc(&b.pos, P * 12)); CK(hipMalloc(&b.vel, P * 12)); CK(hipMalloc(&b.acc, P * 12));
    CK(hipMalloc(&b.mass, P * 4)); CK(hipMalloc(&b.mx, U * 4)); CK(hipMalloc(&b.bounds, U * 8));
    CK(hipMalloc(&b.action, U * 4)); CK(hipMalloc(&b.obs, (size_t)N * D * 4));
    CK(hipMalloc(&b.reward, N * 4)); CK(hipMalloc(&b.energy, N * 4)); CK(hipMalloc(&b.centroid, N * 12));
    CK(hipMalloc(&b.edges, E * 16)); CK(hipMalloc(&b.inc, E * 4)); CK(hipMalloc(&b.inc_off, (P + N) * 2));
    CK(hipMalloc(&b.steps, N * 4)); CK(hipMalloc(&b.contact, P)); CK(hipMalloc(&b.done, N));
    for (void *p : {(void *)b.pos, (void *)b.vel, (void *)b.mass, (void *)b.mx, (void *)b.bounds, (void *)b.action,
                    (void *)b.edges, (void *)b.inc, (void *)b.inc_off, (void *)b.steps})
        (void)p;
    CK(hipMemset(b.pos, 0, P * 12)); CK(hipMemset(b.vel, 0, P * 12)); CK(hipMemset(b.mass, 0, P * 4));
    CK(hipMemset(b.edges, 0, E * 16)); CK(hipMemset(b.inc, 0, E * 4)); CK(hipMemset(b.inc_off, 0, (P + N) * 2));
    const double rd = P * 28.0 + E * 20.0 + U * 16.0 + (P + N) * 2.0 + N * 4.0;
    const double wr = P * 37.0 + (double)N * D * 4 + U * 4.0 + N * 25.0;
    printf("bytes per launch: read %.1f MB, write %.1f MB, total %.1f MB\n", rd / 1e6, wr / 1e6, (rd + wr) / 1e6);
    float4 *src, *dst;
    const size_t nr = (size_t)(rd / 16), nw = (size_t)(wr / 16);
    CK(hipMalloc(&src, nr * 16)); CK(hipMalloc(&dst, nw * 16));
    CK(hipMemset(src, 0, nr * 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    auto timeit = [&](const char *name, auto launch) {
        for (int i = 0; i < 20; i++) launch();
        (void)hipEventRecord(e0);
        const int R = 200;
        for (int i = 0; i < R; i++) launch();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1e3 / R;
        printf("%-8s %7.2f us/launch  %6.2f TB/s\n", name, us, (rd + wr) / (us * 1e-6) / 1e12);
    };
    timeit("copy", [&] { hipLaunchKernelGGL(copy, dim3(4096), dim3(256), 0, 0, src, dst, nr, nw); });
    timeit("skel", [&] { hipLaunchKernelGGL(skel<false>, dim3(N / W), dim3(T), 0, 0, b); });
    timeit("skel_nt", [&] { hipLaunchKernelGGL(skel<true>, dim3(N / W), dim3(T), 0, 0, b); });
    CK(hipDeviceSynchronize());
    return 0;
}
