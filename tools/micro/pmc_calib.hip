// dev: calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 against known byte counts in the access
// patterns of the wavefront kernels (MI355X_MICROARCH.md §HBM: only 16-B/lane streaming reads and
// stores are calibrated there). Each kernel touches a 1 GiB region once (4x the 256 MiB Infinity
// Cache, cold): k_rd32 reads one 32-byte record per lane (the D4 path records), k_rd16 16 B per lane,
// k_rd8 8 B, k_rd4 4 B (item / queue words), k_wr32 writes 32-byte records, k_rd16g gathers 16 B per
// lane at random 128-B-aligned rows (node / primitive loads). Run under
//   rocprofv3 --pmc FETCH_SIZE -- ./pmc_calib   and   rocprofv3 --pmc WRITE_SIZE -- ./pmc_calib
// and divide the counters (kB) by the bytes printed here.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
struct alignas(32) D4 { double x, y, z, w; };
__global__ void k_rd32(const D4* __restrict__ a, double* __restrict__ o, size_t n) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; if (i >= n) return;
    const D4 v = a[i]; if (v.x + v.y + v.z + v.w == 1.2345) o[0] = 1.0;
}
__global__ void k_rd16(const double2* __restrict__ a, double* __restrict__ o, size_t n) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; if (i >= n) return;
    const double2 v = a[i]; if (v.x + v.y == 1.2345) o[0] = 1.0;
}
__global__ void k_rd8(const double* __restrict__ a, double* __restrict__ o, size_t n) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; if (i >= n) return;
    if (a[i] == 1.2345) o[0] = 1.0;
}
__global__ void k_rd4(const unsigned* __restrict__ a, double* __restrict__ o, size_t n) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; if (i >= n) return;
    if (a[i] == 12345u) o[0] = 1.0;
}
__global__ void k_wr32(D4* __restrict__ a, size_t n) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; if (i >= n) return;
    D4 v; v.x = (double)i; v.y = 1.0; v.z = 2.0; v.w = 3.0; a[i] = v;
}
__global__ void k_rd16g(const double2* __restrict__ a, double* __restrict__ o, size_t n_rows, size_t n) {
    size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; if (i >= n) return;
    size_t r = (i * 2654435761ull) % n_rows;            // a scattered 128-B row, 16 B of it
    const double2 v = a[r * 8]; if (v.x + v.y == 1.2345) o[0] = 1.0;
}
int main() {
    const size_t bytes = 1ull << 30;
    char* buf; double* o;
    CK(hipMalloc(&buf, bytes)); CK(hipMalloc(&o, 64));
    CK(hipMemset(buf, 0, bytes));
    CK(hipDeviceSynchronize());
    auto grid = [](size_t n) { return dim3((unsigned)((n + 255) / 256)); };
    size_t n;
    n = bytes / 32; hipLaunchKernelGGL(k_rd32, grid(n), dim3(256), 0, 0, (const D4*)buf, o, n);
    printf("k_rd32  reads %zu bytes\n", n * 32);
    n = bytes / 16; hipLaunchKernelGGL(k_rd16, grid(n), dim3(256), 0, 0, (const double2*)buf, o, n);
    printf("k_rd16  reads %zu bytes\n", n * 16);
    n = bytes / 8; hipLaunchKernelGGL(k_rd8, grid(n), dim3(256), 0, 0, (const double*)buf, o, n);
    printf("k_rd8   reads %zu bytes\n", n * 8);
    n = bytes / 4; hipLaunchKernelGGL(k_rd4, grid(n), dim3(256), 0, 0, (const unsigned*)buf, o, n);
    printf("k_rd4   reads %zu bytes\n", n * 4);
    n = bytes / 32; hipLaunchKernelGGL(k_wr32, grid(n), dim3(256), 0, 0, (D4*)buf, n);
    printf("k_wr32  writes %zu bytes\n", n * 32);
    const size_t rows = bytes / 128; n = rows / 4;       // each touched row once on average (distinct rows: ~78 %)
    hipLaunchKernelGGL(k_rd16g, grid(n), dim3(256), 0, 0, (const double2*)buf, o, rows, n);
    printf("k_rd16g gathers %zu x 16 B from %zu 128-B rows\n", n, rows);
    CK(hipDeviceSynchronize());
    return 0;
}
