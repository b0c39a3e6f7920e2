// Launch / latency floor of a small step (diagnostic, not product; DESIGN §7 "config 2"): what one launch of the
// 4,096-walker Balance-v0 step geometry (128 workgroups x 4 waves, 512 wave tiles) costs with no work, with one
// coalesced load + store per lane, and with a chain of dependent loads, each timed back to back over many launches
// on one stream with HIP events (the per-launch figure bench.py reports for the step itself).
//   empty    : the launch alone
//   load1    : every lane loads one float and stores it (one HBM round trip + the store)
//   chainK   : K dependent loads per lane (the address of each from the previous value), then the store
// build: hipcc --offload-arch=gfx950 -O3 -o build_ablate/launch_floor scripts/launch_floor.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int BLOCKS = 128, THREADS = 256, NLAUNCH = 2000;

__global__ __launch_bounds__(256) void k_empty(float *) {}

__global__ __launch_bounds__(256) void k_load1(const float *__restrict__ in, float *__restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    out[i] = in[i] + 1.0f;
}

template <int K>
__global__ __launch_bounds__(256) void k_chain(const int *__restrict__ nxt, float *__restrict__ out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
    for (int k = 0; k < K; k++) i = nxt[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (float)i;
}

template <typename F>
int timed(const char *name, F launch, hipEvent_t e0, hipEvent_t e1, bool last) {
    for (int i = 0; i < 50; i++) launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < NLAUNCH; i++) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("\"%s_us\": %.3f%s", name, ms * 1e3 / NLAUNCH, last ? "" : ", ");
    return 0;
}

int main() {
    const int n = BLOCKS * THREADS;
    float *in, *out;
    int *nxt;
    CK(hipMalloc(&in, n * sizeof(float)));
    CK(hipMalloc(&out, n * sizeof(float)));
    CK(hipMalloc(&nxt, n * sizeof(int)));
    CK(hipMemset(in, 0, n * sizeof(float)));
    int *h = new int[n];
    for (int i = 0; i < n; i++) h[i] = (int)((i * 2654435761u) % (unsigned)n);   // scattered successor
    CK(hipMemcpy(nxt, h, n * sizeof(int), hipMemcpyHostToDevice));
    delete[] h;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    printf("{\"blocks\": %d, \"threads\": %d, ", BLOCKS, THREADS);
    timed("empty", [&] { hipLaunchKernelGGL(k_empty, dim3(BLOCKS), dim3(THREADS), 0, 0, out); }, e0, e1, false);
    timed("load1", [&] { hipLaunchKernelGGL(k_load1, dim3(BLOCKS), dim3(THREADS), 0, 0, in, out); }, e0, e1, false);
    timed("chain2", [&] { hipLaunchKernelGGL(k_chain<2>, dim3(BLOCKS), dim3(THREADS), 0, 0, nxt, out); }, e0, e1, false);
    timed("chain4", [&] { hipLaunchKernelGGL(k_chain<4>, dim3(BLOCKS), dim3(THREADS), 0, 0, nxt, out); }, e0, e1, false);
    timed("chain8", [&] { hipLaunchKernelGGL(k_chain<8>, dim3(BLOCKS), dim3(THREADS), 0, 0, nxt, out); }, e0, e1, true);
    printf("}\n");
    return 0;
}
