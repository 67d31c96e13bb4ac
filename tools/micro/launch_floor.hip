// dev microbenchmark: the per-launch floor of a bounce-synchronous wavefront on gfx950 -- back-to-back
// launches of kernels whose blocks read a device count and mostly exit (the late bounces of a strong-
// scaled share), with and without a 24 KiB LDS stack per block, for several grid sizes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int LDS>
__global__ __launch_bounds__(256) void k_probe(const unsigned* __restrict__ n, float* __restrict__ out) {
    __shared__ int stk[LDS ? LDS / 4 : 1];
    const unsigned cnt = *n;
    if (blockIdx.x * 256u >= cnt) return;
    const unsigned i = blockIdx.x * 256u + threadIdx.x;
    stk[threadIdx.x] = (int)i;
    __syncthreads();
    if (i < cnt) out[i] = (float)stk[(threadIdx.x + 1) & 255] * 0.5f;
}

template <int LDS>
float run(unsigned grid, unsigned live, const unsigned* d_n, unsigned* d_nw, float* out, int reps) {
    hipMemcpy(d_nw, &live, 4, hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int i = 0; i < 10; ++i) hipLaunchKernelGGL(k_probe<LDS>, dim3(grid), dim3(256), 0, 0, d_n, out);
    hipEventRecord(a, 0);
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k_probe<LDS>, dim3(grid), dim3(256), 0, 0, d_n, out);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms * 1e3f / reps;
}

int main() {
    unsigned* d_n;
    float* out;
    CK(hipMalloc(&d_n, 4));
    CK(hipMalloc(&out, 64u << 20));
    const unsigned grids[] = {1, 64, 256, 1024, 4096, 12600, 50000, 100000};
    const unsigned lives[] = {0, 2048, 30000};
    for (unsigned live : lives)
        for (unsigned g : grids) {
            if (live > g * 256u) continue;
            const float t0 = run<0>(g, live, d_n, d_n, out, 200);
            const float t24 = run<24576>(g, live, d_n, d_n, out, 200);
            printf("grid %6u blocks, live %6u threads: %7.2f us/launch (no LDS)  %7.2f us/launch (24 KiB LDS)\n", g, live, t0, t24);
        }
    return 0;
}
