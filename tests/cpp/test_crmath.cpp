// rs_crmath.h (host build) against libquadmath's 113-bit sin / cos / pow rounded to double.
// usage: test_crmath N  -> prints mismatch counts per family; exit 1 if any.
#include <quadmath.h>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../../include/rs_crmath.h"

static double u01(std::mt19937_64& g) { return (double)(g() >> 11) * 0x1p-53; }

int main(int argc, char** argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    std::mt19937_64 g(7);
    long bad[6] = {0, 0, 0, 0, 0, 0};
    int shown = 0;
    for (long i = 0; i < n; ++i) {
        // the cosine-direction argument 2 pi r1 (vec3.rs:100-111)
        const double a = 2.0 * 3.141592653589793 * u01(g);
        // checker arguments scale * p (checker.rs:21-30), |p| up to 1e4
        const double b = 10.0 * (u01(g) * 2e4 - 1e4);
        // the Phong lobe r2 = gen^(1/(e+1)) (vec3.rs:115-126), e in [0, 1000]
        const double x = u01(g), y = 1.0 / (u01(g) * 1000.0 + 1.0);
        // generic pow: x in (0, 4), y in (-8, 8)
        const double x2 = u01(g) * 4.0, y2 = u01(g) * 16.0 - 8.0;
        double s, c;
        rs_cr::sincos_cr(a, &s, &c);
        if (s != (double)sinq(a)) { ++bad[0]; if (shown++ < 5) printf("sin(%a) %a vs %a\n", a, s, (double)sinq(a)); }
        if (c != (double)cosq(a)) ++bad[1];
        rs_cr::sincos_cr(b, &s, &c);
        if (s != (double)sinq(b)) ++bad[2];
        if (c != (double)cosq(b)) ++bad[3];
        const double p = rs_cr::pow_cr(x, y);
        if (p != (double)powq(x, y)) { ++bad[4]; if (shown++ < 10) printf("pow(%a, %a) %a vs %a\n", x, y, p, (double)powq(x, y)); }
        if (x2 > 0 && rs_cr::pow_cr(x2, y2) != (double)powq(x2, y2)) ++bad[5];
    }
    // checker sign: sin3_negative == (sin_cr(a) sin_cr(b) sin_cr(c) < 0), incl. zeros
    long bad_sign = 0;
    for (long i = 0; i < n / 4; ++i) {
        double v[3];
        for (double& t : v) {
            const uint64_t r = g();
            t = (r & 15) == 0 ? ((r & 16) ? 0.0 : -0.0) : 20.0 * (u01(g) * 2e4 - 1e4);
        }
        const bool ref = rs_cr::sin_cr(v[0]) * rs_cr::sin_cr(v[1]) * rs_cr::sin_cr(v[2]) < 0.0;
        bad_sign += ref != rs_cr::sin3_negative(v[0], v[1], v[2]);
    }
    bad[5] += bad_sign;
    // special values
    long spec = 0;
    double s, c;
    rs_cr::sincos_cr(0.0, &s, &c); spec += !(s == 0.0 && !std::signbit(s) && c == 1.0);
    rs_cr::sincos_cr(-0.0, &s, &c); spec += !(s == 0.0 && std::signbit(s) && c == 1.0);
    rs_cr::sincos_cr(INFINITY, &s, &c); spec += !(s != s && c != c);
    spec += rs_cr::pow_cr(0.0, 0.5) != 0.0;
    spec += rs_cr::pow_cr(1.0, 123.0) != 1.0;
    spec += rs_cr::pow_cr(0.25, 0.5) != 0.5;
    spec += rs_cr::pow_cr(0.7, 1.0) != 0.7;
    printf("n=%ld mismatches vs quad: sin[0,2pi) %ld cos %ld sin[-1e5,1e5) %ld cos %ld pow(gen,1/(e+1)) %ld pow(generic) %ld specials %ld\n",
           n, bad[0], bad[1], bad[2], bad[3], bad[4], bad[5], spec);
    return (bad[0] + bad[1] + bad[2] + bad[3] + bad[4] + bad[5] + spec) ? 1 : 0;
}
