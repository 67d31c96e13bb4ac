// dev: how often do ocml's double sin / cos / sincos / pow differ from glibc's (the reference's
// libm) on the inputs the path tracer feeds them?
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <random>
#include <vector>

__global__ void k(const double* x, const double* e, double* s, double* c, double* ss, double* cc, double* p, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    s[i] = sin(x[i]);
    c[i] = cos(x[i]);
    double a, b;
    sincos(x[i], &a, &b);
    ss[i] = a; cc[i] = b;
    p[i] = pow(e[i], 1.0 / (e[i] * 300.0 + 1.0));
}

int main() {
    const int n = 1 << 24;
    std::vector<double> x(n), e(n);
    std::mt19937_64 g(1);
    for (int i = 0; i < n; ++i) {
        double r = (double)(g() >> 11) * 0x1p-53;
        x[i] = (i % 2) ? 2.0 * 3.141592653589793 * r : 10.0 * ((double)(g() >> 11) * 0x1p-53 * 2000.0 - 1000.0);
        e[i] = (double)(g() >> 11) * 0x1p-53;
    }
    double *dx, *de, *ds, *dc, *dss, *dcc, *dp;
    hipMalloc(&dx, n * 8); hipMalloc(&de, n * 8); hipMalloc(&ds, n * 8); hipMalloc(&dc, n * 8);
    hipMalloc(&dss, n * 8); hipMalloc(&dcc, n * 8); hipMalloc(&dp, n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    hipMemcpy(de, e.data(), n * 8, hipMemcpyHostToDevice);
    k<<<n / 256, 256>>>(dx, de, ds, dc, dss, dcc, dp, n);
    std::vector<double> s(n), c(n), ss(n), cc(n), p(n);
    hipMemcpy(s.data(), ds, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(c.data(), dc, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(ss.data(), dss, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(cc.data(), dcc, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(p.data(), dp, n * 8, hipMemcpyDeviceToHost);
    long bs[2] = {0, 0}, bc[2] = {0, 0}, bss[2] = {0, 0}, bcc[2] = {0, 0}, bp = 0;
    int shown = 0;
    for (int i = 0; i < n; ++i) {
        int r = i % 2;  // 1: [0, 2pi) (cosine direction), 0: [-1e4, 1e4) (checker)
        if (s[i] != std::sin(x[i])) { ++bs[r]; if (shown < 5) { printf("sin(%.17g): gpu %.17g glibc %.17g\n", x[i], s[i], std::sin(x[i])); ++shown; } }
        if (c[i] != std::cos(x[i])) ++bc[r];
        if (ss[i] != std::sin(x[i])) ++bss[r];
        if (cc[i] != std::cos(x[i])) ++bcc[r];
        if (p[i] != std::pow(e[i], 1.0 / (e[i] * 300.0 + 1.0))) ++bp;
    }
    printf("n=%d per range\n[0,2pi): sin %ld cos %ld sincos.s %ld sincos.c %ld\n[-1e4,1e4): sin %ld cos %ld sincos.s %ld sincos.c %ld\npow %ld of %d\n",
           n / 2, bs[1], bc[1], bss[1], bcc[1], bs[0], bc[0], bss[0], bcc[0], bp, n);
    return 0;
}
