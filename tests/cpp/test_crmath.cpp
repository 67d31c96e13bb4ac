// rs_crmath.h (host build) against libquadmath's 113-bit sin / cos / pow rounded to double.
// usage: test_crmath N  -> prints mismatch counts per family; exit 1 if any.
#include <quadmath.h>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <cmath>

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
    // log of a uniform draw (ConstantMedium, medium/constant.rs:63); atan2 / asin of unit-vector
    // components (Sphere::uv, sphere.rs:64-71) and of generic arguments
    long bad_log = 0, bad_atan2 = 0, bad_asin = 0;
    for (long i = 0; i < n; ++i) {
        const double u = (double)g() * 0x1p-64;
        if (u > 0.0 && rs_cr::log_cr(u) != (double)logq(u)) { ++bad_log; if (shown++ < 15) printf("log(%a) %a vs %a\n", u, rs_cr::log_cr(u), (double)logq(u)); }
        const double x = u01(g) * 2.0 - 1.0, y = u01(g) * 2.0 - 1.0, z = u01(g) * 2.0 - 1.0;
        const double l = std::sqrt(x * x + y * y + z * z);
        if (l == 0.0 || l > 1.0) continue;
        const double px = x / l, py = y / l, pz = z / l;
        if (rs_cr::atan2_cr(-pz, px) != (double)atan2q(-pz, px)) { ++bad_atan2; if (shown++ < 20) printf("atan2(%a, %a) %a vs %a\n", -pz, px, rs_cr::atan2_cr(-pz, px), (double)atan2q(-pz, px)); }
        if (rs_cr::asin_cr(py) != (double)asinq(py)) { ++bad_asin; if (shown++ < 25) printf("asin(%a) %a vs %a\n", py, rs_cr::asin_cr(py), (double)asinq(py)); }
        const double ga = (u01(g) - 0.5) * std::ldexp(1.0, (int)(g() % 40) - 20), gb = (u01(g) - 0.5) * std::ldexp(1.0, (int)(g() % 40) - 20);
        if (rs_cr::atan2_cr(ga, gb) != (double)atan2q(ga, gb)) ++bad_atan2;
        const double ys = std::ldexp(u01(g), -(int)(g() % 30));
        if (rs_cr::asin_cr(ys) != (double)asinq(ys)) ++bad_asin;
    }
    const double edge[] = {1.0, -1.0, 0x1.fffffffffffffp-1, 0.5, -0.5, 0x1p-30, 0x1p-1000};
    for (double e : edge) bad_asin += rs_cr::asin_cr(e) != (double)asinq(e);
    bad_log += rs_cr::log_cr(1.0) != 0.0;
    bad_log += rs_cr::log_cr(0.0) != -INFINITY;
    bad_atan2 += !(rs_cr::atan2_cr(0.0, -1.0) == (double)atan2q(0.0, -1.0) && rs_cr::atan2_cr(-0.0, 1.0) == 0.0 &&
                   std::signbit(rs_cr::atan2_cr(-0.0, 1.0)));
    bad_atan2 += rs_cr::atan2_cr(1.0, 0.0) != (double)atan2q(1.0, 0.0);
    printf("n=%ld mismatches vs quad: log %ld atan2 %ld asin %ld\n", n, bad_log, bad_atan2, bad_asin);
    bad[5] += bad_log + bad_atan2 + bad_asin;
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
