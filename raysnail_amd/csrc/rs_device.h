// rs_device.h — device-side path tracing primitives for gfx950 (MI355X).
//
// Arithmetic mirrors raysnail's f64 semantics operation by operation (build with
// -ffp-contract=off; explicit fma() exactly where the reference calls mul_add):
//   Vec3::dot / length_squared via mul_add           src/prelude/vec3.rs:152-155,177-179
//   Vec3::unit = v * (1/len)                         src/prelude/vec3.rs:192-194,486-492
//   Ray::at per-axis mul_add                         src/prelude/ray.rs:21-31
//   AABB::hit slab test                              src/prelude/aabb.rs:20-38
// The per-primitive / per-material functions cite their reference lines below.
#pragma once
#include "../../include/rs_crmath.h"
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "rs_layout.h"
#include "../../include/raysnail_hip.h"

#define RS_REJECTION_CAP 4096
#define RS_INF __builtin_huge_val()
#define RS_FMAX 1.7976931348623157e308
#define RS_PI 3.14159265358979323846

namespace rs {

// ------------------------------------------------------------------ Vec3 ----
struct V3 { double x, y, z; };
__device__ __forceinline__ V3 v3(double x, double y, double z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ V3 operator*(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ V3 operator*(double s, V3 a) { return v3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ double dot(V3 a, V3 b) { return fma(a.z, b.z, fma(a.x, b.x, a.y * b.y)); }
__device__ __forceinline__ double len2(V3 a) { return fma(a.z, a.z, fma(a.x, a.x, a.y * a.y)); }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ V3 vdiv(V3 a, double s) { double inv = 1.0 / s; return a * inv; }
__device__ __forceinline__ V3 unit(V3 a) { return vdiv(a, sqrt(len2(a))); }
__device__ __forceinline__ double comp(V3 a, int i) { return i == 0 ? a.x : (i == 1 ? a.y : a.z); }
__device__ __forceinline__ V3 ld3(const double* p) { return v3(p[0], p[1], p[2]); }
// vec3.rs:171-173 / material/mod.rs:75-81: d - n * (2 * d.n)
__device__ __forceinline__ V3 reflect_v(V3 d, V3 n) { return d - n * (2.0 * dot(d, n)); }

// key: the medium key of the segment (rs_medium_uniform); only read when the scene has media
struct Ray { V3 o, d; double time; uint64_t key; };
__device__ __forceinline__ V3 ray_at(const Ray& r, double t) {
    return v3(fma(r.d.x, t, r.o.x), fma(r.d.y, t, r.o.y), fma(r.d.z, t, r.o.z));
}

// ------------------------------------------------------------------ RNG ----
// rand_xorshift 0.3.0 XorShiftRng seeded by rand_core 0.6 seed_from_u64 (src/prelude/random.rs:109-145)
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

struct Rng {
    uint32_t x, y, z, w;
    __device__ __forceinline__ void seed_from_u64(uint64_t st) {
        uint32_t s[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            st = st * 6364136223846793005ULL + 11634580027462260723ULL;
            uint32_t xs = (uint32_t)(((st >> 18) ^ st) >> 27);
            uint32_t rot = (uint32_t)(st >> 59);
            s[i] = (xs >> rot) | (xs << ((32u - rot) & 31u));
        }
        if ((s[0] | s[1] | s[2] | s[3]) == 0u) { s[0] = s[1] = s[2] = s[3] = 0x0BAD5EEDu; }
        x = s[0]; y = s[1]; z = s[2]; w = s[3];
    }
    __device__ __forceinline__ uint32_t next_u32() {
        uint32_t t = x ^ (x << 11);
        x = y; y = z; z = w;
        w = w ^ (w >> 19) ^ (t ^ (t >> 8));
        return w;
    }
    // next_u64 as f64 / u64::MAX as f64 (== 2^64): in [0, 1] inclusive
    __device__ __forceinline__ double gen() {
        uint64_t lo = next_u32();
        uint64_t hi = next_u32();
        return (double)((hi << 32) | lo) * 0x1p-64;
    }
    __device__ __forceinline__ double range(double a, double b) { return a + gen() * (b - a); }
    // the segment's medium key: a hash of the state, not a draw (the stream is not advanced)
    __device__ __forceinline__ uint64_t medium_key() const {
        return splitmix64((((uint64_t)y << 32) | x) ^ splitmix64(((uint64_t)w << 32) | z));
    }
};
// ConstantMedium's Random::normal() (constant.rs:63) for medium handle h: uniform in [0, 1]
__device__ __forceinline__ double medium_uniform(uint64_t key, int h) {
    return (double)splitmix64(key ^ splitmix64(0x6d656469756d2121ULL + (uint64_t)(uint32_t)h)) * 0x1p-64;
}

// ------------------------------------------------------------------ hit record ----
struct Hit {
    V3 p, n;
    double t1, t2;
    double u, v;   // written only when the scene reads them (the `uv` flag of the hit functions: rich
                   // scene mode with an Image texture); left unset otherwise, so they cost nothing
    int32_t mat;
    int32_t outside;
};

// ------------------------------------------------------------------ shapes ----
__device__ __forceinline__ bool in_range(double t, double a, double b) { return a <= t && t < b; }

// hit.rs:32-53 HitRecord::new with the object's normal already computed
__device__ __forceinline__ void finish_rec(Hit& h, const Ray& r, double t1, double t2, V3 nrm, int32_t mat) {
    h.p = ray_at(r, t1);
    h.t1 = t1; h.t2 = t2; h.mat = mat;
    bool outside = dot(r.d, nrm) < 0.0;
    h.n = outside ? nrm : -nrm;
    h.outside = outside;
}

// sphere.rs:83-109. Returns the chosen t (t1 or t2 per the reference) or -1 sentinel via ok.
__device__ __forceinline__ bool sphere_t(const DSphere& s, const Ray& r, double tmin, double tmax, double& t, double& t2o) {
    V3 cc = ld3(s.c) + ld3(s.v) * r.time;
    V3 l = r.o - cc;
    double half_b = dot(r.d, l);
    double a = len2(r.d);
    double c = len2(l) - s.r2;
    double delta = half_b * half_b - a * c;
    if (delta < 0.0) return false;
    double sq = sqrt(delta);
    double t1 = (-half_b - sq) / a;
    double t2 = (-half_b + sq) / a;
    t2o = t2;
    if (in_range(t1, tmin, tmax)) { t = t1; return true; }
    if (in_range(t2, tmin, tmax)) { t = t2; return true; }
    return false;
}
__device__ __forceinline__ V3 sphere_normal(const DSphere& s, V3 p) { return vdiv(p - ld3(s.c), s.r); }

// sphere.rs:64-71 (static center; correctly rounded atan2 / asin, rs_crmath.h)
// (out of line: only image-textured scenes call it; keeps the hot kernels' register budget)
__device__ __noinline__ void sphere_uv(const DSphere& s, V3 point, double& u, double& v) {
    const V3 p = unit(point - ld3(s.c));
    const double phi = rs_cr::atan2_cr(-p.z, p.x);
    const double theta = rs_cr::asin_cr(p.y);
    u = phi / 2.0 / RS_PI + 0.5;
    v = theta / RS_PI + 0.5;
}

__device__ __forceinline__ bool sphere_hit(const DSphere& s, int32_t mat, const Ray& r, double tmin, double tmax, Hit& h,
                                           int uv = 0) {
    double t, t2;
    if (!sphere_t(s, r, tmin, tmax, t, t2)) return false;
    V3 p = ray_at(r, t);
    finish_rec(h, r, t, t2, sphere_normal(s, p), mat);
    if (uv) sphere_uv(s, h.p, h.u, h.v);
    return true;
}

// Sphere::hit's record (sphere_hit) for the root t the traversal already chose (sphere_t's arithmetic: the
// same t bit for bit): the point, the normal from the static center, the front-face flip. t2 is left at
// RS_FMAX: only CSG decisions read it, and the spheres scene mode that uses this has none.
__device__ __forceinline__ void sphere_rec_at(const DSphere& s, int32_t mat, const Ray& r, double t, Hit& h) {
    const V3 p = ray_at(r, t);
    finish_rec(h, r, t, RS_FMAX, sphere_normal(s, p), mat);
}

// rect.rs:101-120
__device__ __forceinline__ bool rect_hit_raw(int ax0, int ax1, int ax2, double k, double a0, double a1, double b0, double b1,
                                             int32_t mat, const Ray& r, double tmin, double tmax, Hit& h, int uv = 0) {
    double t1 = (k - comp(r.o, ax2)) / comp(r.d, ax2);
    if (!in_range(t1, tmin, tmax)) return false;
    double a = fma(t1, comp(r.d, ax0), comp(r.o, ax0));
    if (a < a0 || a > a1) return false;
    double b = fma(t1, comp(r.d, ax1), comp(r.o, ax1));
    if (b < b0 || b > b1) return false;
    V3 n = v3(ax2 == 0 ? 1.0 : 0.0, ax2 == 1 ? 1.0 : 0.0, ax2 == 2 ? 1.0 : 0.0);
    finish_rec(h, r, t1, RS_FMAX, n, mat);
    if (uv) { h.u = (a - a0) / (a1 - a0); h.v = (b - b0) / (b1 - b0); }  // rect.rs:94-99 (a_len, b_len)
    return true;
}

// Box::hit's (t1, t2) alone (box.rs:125-149): the first two face hits in face order; one -> (t, MAX),
// two -> (nearer, farther). What the traversal and the CSG decisions read (the record: box_hit).
__device__ __forceinline__ bool box_t(const DBox& b, const Ray& r, double tmin, double tmax, double& t1o, double& t2o) {
    double ta = 0.0, tb = 0.0;
    int n = 0;
#pragma unroll
    for (int f = 0; f < 6; ++f) {
        int ax0, ax1, ax2; double k, a0, a1, b0, b1;
        if (f < 2)      { ax0 = 0; ax1 = 1; ax2 = 2; k = f == 0 ? b.mn[2] : b.mx[2]; a0 = b.mn[0]; a1 = b.mx[0]; b0 = b.mn[1]; b1 = b.mx[1]; }
        else if (f < 4) { ax0 = 1; ax1 = 2; ax2 = 0; k = f == 2 ? b.mn[0] : b.mx[0]; a0 = b.mn[1]; a1 = b.mx[1]; b0 = b.mn[2]; b1 = b.mx[2]; }
        else            { ax0 = 0; ax1 = 2; ax2 = 1; k = f == 4 ? b.mn[1] : b.mx[1]; a0 = b.mn[0]; a1 = b.mx[0]; b0 = b.mn[2]; b1 = b.mx[2]; }
        if (n < 2) {
            const double t = (k - comp(r.o, ax2)) / comp(r.d, ax2);
            if (in_range(t, tmin, tmax)) {
                const double a = fma(t, comp(r.d, ax0), comp(r.o, ax0));
                const double bb = fma(t, comp(r.d, ax1), comp(r.o, ax1));
                if (!(a < a0 || a > a1) && !(bb < b0 || bb > b1)) {
                    if (n == 0) ta = t; else tb = t;
                    ++n;
                }
            }
        }
    }
    if (n == 0) return false;
    if (n == 1) { t1o = ta; t2o = RS_FMAX; return true; }
    if (ta < tb) { t1o = ta; t2o = tb; } else { t1o = tb; t2o = ta; }
    return true;
}

__device__ __forceinline__ bool rect_t(const DRect& R, const Ray& r, double tmin, double tmax, double& t1) {
    const double t = (R.k - comp(r.o, R.ax2)) / comp(r.d, R.ax2);
    if (!in_range(t, tmin, tmax)) return false;
    const double a = fma(t, comp(r.d, R.ax0), comp(r.o, R.ax0));
    if (a < R.a0 || a > R.a1) return false;
    const double b = fma(t, comp(r.d, R.ax1), comp(r.o, R.ax1));
    if (b < R.b0 || b > R.b1) return false;
    t1 = t;
    return true;
}

// box.rs:125-149; faces in the order built by box.rs:55-105
__device__ bool box_hit(const DBox& b, int32_t mat, const Ray& r, double tmin, double tmax, Hit& h, int uv = 0) {
    Hit h0, h1;  // the first two face hits in face order (two named records: no scratch array)
    int n = 0;
#pragma unroll
    for (int f = 0; f < 6; ++f) {
        int ax0, ax1, ax2; double k, a0, a1, b0, b1;
        if (f < 2)      { ax0 = 0; ax1 = 1; ax2 = 2; k = f == 0 ? b.mn[2] : b.mx[2]; a0 = b.mn[0]; a1 = b.mx[0]; b0 = b.mn[1]; b1 = b.mx[1]; }
        else if (f < 4) { ax0 = 1; ax1 = 2; ax2 = 0; k = f == 2 ? b.mn[0] : b.mx[0]; a0 = b.mn[1]; a1 = b.mx[1]; b0 = b.mn[2]; b1 = b.mx[2]; }
        else            { ax0 = 0; ax1 = 2; ax2 = 1; k = f == 4 ? b.mn[1] : b.mx[1]; a0 = b.mn[0]; a1 = b.mx[0]; b0 = b.mn[2]; b1 = b.mx[2]; }
        if (n < 2) {
            Hit t;
            if (rect_hit_raw(ax0, ax1, ax2, k, a0, a1, b0, b1, mat, r, tmin, tmax, t, uv)) {
                if (n == 0) h0 = t; else h1 = t;
                ++n;
            }
        }
    }
    if (n == 0) return false;
    if (n == 1) { h = h0; return true; }
    // with_normal (hit.rs:55-67): outside = true, normal as recorded by the face
    if (h0.t1 < h1.t1) { h = h0; h.t2 = h1.t1; }
    else { h = h1; h.t2 = h0.t1; }
    h.outside = 1;
    return true;
}
__device__ __forceinline__ bool box_contains(const DBox& b, V3 p) {
    return p.x >= b.mn[0] && p.x <= b.mx[0] && p.y >= b.mn[1] && p.y <= b.mx[1] && p.z >= b.mn[2] && p.z <= b.mx[2];
}

// quadric.rs:67-100
__device__ V3 quadric_normal(const DQuadric& Q, V3 p) {
    const double* q = Q.q;  // qa qb qc qd qe qf qg qh qi qj
    double x = 2.0 * q[0] * p.x + q[1] * p.y + q[2] * p.z + q[3];
    double y = q[1] * p.x + 2.0 * q[4] * p.y + q[5] * p.z + q[6];
    double z = q[2] * p.x + q[5] * p.y + 2.0 * q[7] * p.z + q[8];
    V3 rr = v3(x, y, z);
    double len = sqrt(len2(rr));
    if (len == 0.0) return v3(1.0, 0.0, 0.0);
    return vdiv(rr, len);
}
// Quadric::hit's (t1, t2) alone (quadric.rs:112-182; the record: quadric_hit)
__device__ __forceinline__ bool quadric_t(const DQuadric& Q, const Ray& r, double tmin, double tmax, double& t1, double& t2) {
    const double* q = Q.q;
    const double qa = q[0], qb = q[1], qc = q[2], qd = q[3], qe = q[4], qf = q[5], qg = q[6], qh = q[7], qi = q[8], qj = q[9];
    double xo = r.o.x, yo = r.o.y, zo = r.o.z, xd = r.d.x, yd = r.d.y, zd = r.d.z;
    double a = xd * (qa * xd + qb * yd + qc * zd) + yd * (qe * yd + qf * zd) + zd * qh * zd;
    double b = xd * (qa * xo + 0.5 * (qb * yo + qc * zo + qd)) + yd * (qe * yo + 0.5 * (qb * xo + qf * zo + qg)) +
               zd * (qh * zo + 0.5 * (qc * xo + qf * yo + qi));
    double c = xo * (qa * xo + qb * yo + qc * zo + qd) + yo * (qe * yo + qf * zo + qg) + zo * (qh * zo + qi) + qj;
    if (a == 0.0) {
        if (b == 0.0) return false;
        t1 = -0.5 * c / b;
        if (!in_range(t1, tmin, tmax)) return false;
        t2 = RS_FMAX;
        return true;
    }
    double d = b * b - a * c;
    if (d <= 0.0) return false;
    double dr = sqrt(d);
    double r1 = (-b - dr) / a;
    double r2 = (-b + dr) / a;
    if (in_range(r1, tmin, tmax)) { t1 = r1; t2 = r2; return true; }
    if (in_range(r2, tmin, tmax)) { t1 = r2; t2 = RS_FMAX; return true; }
    return false;
}

// quadric.rs:112-182
__device__ bool quadric_hit(const DQuadric& Q, int32_t mat, const Ray& r, double tmin, double tmax, Hit& h, int uv = 0) {
    const double* q = Q.q;
    const double qa = q[0], qb = q[1], qc = q[2], qd = q[3], qe = q[4], qf = q[5], qg = q[6], qh = q[7], qi = q[8], qj = q[9];
    double xo = r.o.x, yo = r.o.y, zo = r.o.z, xd = r.d.x, yd = r.d.y, zd = r.d.z;
    double a = xd * (qa * xd + qb * yd + qc * zd) + yd * (qe * yd + qf * zd) + zd * qh * zd;
    double b = xd * (qa * xo + 0.5 * (qb * yo + qc * zo + qd)) + yd * (qe * yo + 0.5 * (qb * xo + qf * zo + qg)) +
               zd * (qh * zo + 0.5 * (qc * xo + qf * yo + qi));
    double c = xo * (qa * xo + qb * yo + qc * zo + qd) + yo * (qe * yo + qf * zo + qg) + zo * (qh * zo + qi) + qj;
    double t1, t2;
    if (a == 0.0) {
        if (b == 0.0) return false;
        t1 = -0.5 * c / b;
        if (!in_range(t1, tmin, tmax)) return false;
        t2 = RS_FMAX;
    } else {
        double d = b * b - a * c;
        if (d <= 0.0) return false;
        double dr = sqrt(d);
        double r1 = (-b - dr) / a;
        double r2 = (-b + dr) / a;
        if (in_range(r1, tmin, tmax)) { t1 = r1; t2 = r2; }
        else if (in_range(r2, tmin, tmax)) { t1 = r2; t2 = RS_FMAX; }
        else return false;
    }
    V3 p = ray_at(r, t1);
    finish_rec(h, r, t1, t2, quadric_normal(Q, p), mat);
    if (uv) { h.u = 0.0; h.v = 0.0; }  // Quadric::uv (quadric.rs:106-110)
    return true;
}
__device__ __forceinline__ bool quadric_contains(const DQuadric& Q, V3 p) {  // quadric.rs:184-189
    const double* q = Q.q;
    return (p.x * (q[0] * p.x + q[1] * p.y + q[3]) + p.y * (q[4] * p.y + q[5] * p.z + q[6]) +
            p.z * (q[7] * p.z + q[2] * p.x + q[8]) + q[9]) <= 0.0;
}

// triangle_mesh.rs:85-131
// tri_hit's accept test alone (the traversal's leaf test; the winner's record is recomputed).
// TRI: DTri or the leaf-ordered LTri (same p0 / a..f fields). (Skipping the divisions for lanes whose
// quotient sign / magnitude already rejects was measured slower: under divergence the wave still runs
// the division for its other lanes, and the extra registers spilled the flat-scene extend.)
template <typename TRI>
__device__ __forceinline__ bool tri_t(const TRI& T, const Ray& r, double tmin, double tmax, double& t_out) {
    double g = r.d.x, hh = r.d.y, i = r.d.z;
    double j = T.p0[0] - r.o.x, k = T.p0[1] - r.o.y, l = T.p0[2] - r.o.z;
    double eihf = T.e * i - hh * T.f;
    double gfdi = g * T.f - T.d * i;
    double dheg = T.d * hh - T.e * g;
    double denom = T.a * eihf + T.b * gfdi + T.c * dheg;
    // (Rejecting before the divisions where the sign / magnitude of the numerator already decides
    // the quotient's test measured slower on C5, 49.5 vs 47.8 ms: the branches cost more than the
    // divisions under divergence.)
    const double nb = j * eihf + k * gfdi + l * dheg;
    double beta = nb / denom;
    if (beta < 0.0 || beta >= 1.0) return false;
    double akjb = T.a * k - j * T.b;
    double jcal = j * T.c - T.a * l;
    double blkc = T.b * l - k * T.c;
    const double ng = i * akjb + hh * jcal + g * blkc;
    double gamma = ng / denom;
    if (gamma <= 0.0 || beta + gamma >= 1.0) return false;
    double t = -(T.f * akjb + T.e * jcal + T.d * blkc) / denom;
    if (!(t >= tmin && t <= tmax)) return false;
    t_out = t;
    return true;
}

__device__ bool tri_hit(const DTri& T, int32_t mat, const Ray& r, double tmin, double tmax, Hit& h, int uv = 0) {
    double g = r.d.x, hh = r.d.y, i = r.d.z;
    double j = T.p0[0] - r.o.x, k = T.p0[1] - r.o.y, l = T.p0[2] - r.o.z;
    double eihf = T.e * i - hh * T.f;
    double gfdi = g * T.f - T.d * i;
    double dheg = T.d * hh - T.e * g;
    double denom = T.a * eihf + T.b * gfdi + T.c * dheg;
    double beta = (j * eihf + k * gfdi + l * dheg) / denom;
    if (beta < 0.0 || beta >= 1.0) return false;
    double akjb = T.a * k - j * T.b;
    double jcal = j * T.c - T.a * l;
    double blkc = T.b * l - k * T.c;
    double gamma = (i * akjb + hh * jcal + g * blkc) / denom;
    if (gamma <= 0.0 || beta + gamma >= 1.0) return false;
    double t = -(T.f * akjb + T.e * jcal + T.d * blkc) / denom;
    if (!(t >= tmin && t <= tmax)) return false;
    V3 n = ld3(T.n0) * (1.0 - beta - gamma) + ld3(T.n1) * beta + ld3(T.n2) * gamma;
    h.p = ray_at(r, t);
    h.n = n; h.t1 = t; h.t2 = RS_FMAX; h.mat = mat; h.outside = 1;   // with_normal
    if (uv) { h.u = 0.0; h.v = 0.0; }                                    // Triangle::uv (:80-82)
    return true;
}

// transform.rs:133-157 with vecmath row_mat4_transform
__device__ __forceinline__ V3 mat_apply(const DMat34& M, V3 p, double w) {
    const double (*m)[4] = M.m;
    return v3(m[0][0] * p.x + m[0][1] * p.y + m[0][2] * p.z + m[0][3] * w,
              m[1][0] * p.x + m[1][1] * p.y + m[1][2] * p.z + m[1][3] * w,
              m[2][0] * p.x + m[2][1] * p.y + m[2][2] * p.z + m[2][3] * w);
}
__device__ __forceinline__ V3 tf_forward(const DScene& S, const DXform& X, int n, V3 p, double w) {
    for (int i = 0; i < n; ++i) p = mat_apply(S.tf_fwd[X.first + i], p, w);
    return p;
}
__device__ __forceinline__ V3 tf_inverse(const DScene& S, const DXform& X, int n, V3 p, double w) {
    for (int i = n - 1; i >= 0; --i) p = mat_apply(S.tf_inv[X.first + i], p, w);
    return p;
}
// a ray's origin (w = 1) and direction (w = 0) through the same inverse matrices in one pass: the
// same products as two tf_inverse calls, each matrix loaded once (the nested-object tests of the
// nest-2 extend: 162 -> 127 VGPRs for Obj<2>::hit_t with the Difference change below)
__device__ __forceinline__ void tf_inverse_ray(const DScene& S, const DXform& X, int n, V3& o, V3& d) {
    for (int i = n - 1; i >= 0; --i) {
        const DMat34 M = S.tf_inv[X.first + i];
        o = mat_apply(M, o, 1.0);
        d = mat_apply(M, d, 0.0);
    }
}

// ------------------------------------------------------------------ objects (nested) ----
// Obj<L, R>: nested-object dispatch L levels deep; R = 1 in the rich scene mode (ConstantMedium,
// records with (u, v)), 0 elsewhere, so the common kernels carry none of that code.
template <int L, int R> struct Obj;

// What the traversal and the CSG decisions read of a hit() record: t1, t2 and the point (a TfFacade
// record's point is mapped forward, so it is not always ray.at(t1)). hit_t decides exactly what hit()
// decides and returns these fields bit for bit; hit() builds the full record of the one object that
// won (CSG: the winning child's own hit()), so no Hit records are live during the decisions.
struct HitT { double t1, t2; V3 p; };

template <int R> struct Obj<-1, R> {
    static __device__ bool hit(const DScene&, int, const Ray&, double, double, Hit&) { return false; }
    static __device__ bool hit_t(const DScene&, int, const Ray&, double, double, HitT&) { return false; }
    static __device__ bool contains(const DScene&, int, V3) { return false; }
    static __device__ V3 random(const DScene&, int, V3, Rng&) { return v3(1.0, 0.0, 0.0); }
};

template <int L, int R> struct Obj {
    // one call site of the level below per query (composite_t) where the levels are inlined; the
    // generic / rich mode's levels are calls, which keep the per-child sites (composite_t_calls)
    static constexpr bool kOneSite = L <= 2 && R == 0;
    // inlined in the scene modes with at most two nesting levels (no call frames and no spills in
    // their traversal loops); the generic mode's up-to-4-level copies stay calls (code size)
    static __device__ __forceinline__ bool hit_t(const DScene& S, int pi, const Ray& r, double tmin, double tmax, HitT& h) {
        if constexpr (L <= 2 && R == 0) return hit_t_body(S, pi, r, tmin, tmax, h);
        else return hit_t_call(S, pi, r, tmin, tmax, h);
    }
    static __device__ __noinline__ bool hit_t_call(const DScene& S, int pi, const Ray& r, double tmin, double tmax, HitT& h) {
        return hit_t_body(S, pi, r, tmin, tmax, h);
    }
    static __device__ __forceinline__ bool hit_t_body(const DScene& S, int pi, const Ray& r, double tmin, double tmax,
                                                     HitT& h) {
        const DPrim P = S.prims[pi];
        switch (P.kind) {
        case PK_SPHERE: {
            double t, t2;
            if (!sphere_t(S.spheres[P.idx], r, tmin, tmax, t, t2)) return false;
            h.t1 = t; h.t2 = t2; h.p = ray_at(r, t);
            return true;
        }
        case PK_RECT:
            if (!rect_t(S.rects[P.idx], r, tmin, tmax, h.t1)) return false;
            h.t2 = RS_FMAX; h.p = ray_at(r, h.t1);
            return true;
        case PK_BOX:
            if (!box_t(S.boxes[P.idx], r, tmin, tmax, h.t1, h.t2)) return false;
            h.p = ray_at(r, h.t1);
            return true;
        case PK_QUADRIC:
            if (!quadric_t(S.quadrics[P.idx], r, tmin, tmax, h.t1, h.t2)) return false;
            h.p = ray_at(r, h.t1);
            return true;
        case PK_TRIANGLE:
            if (!tri_t(S.tris[P.idx], r, tmin, tmax, h.t1)) return false;
            h.t2 = RS_FMAX; h.p = ray_at(r, h.t1);
            return true;
        case PK_AND:    // csg/intersection.rs:58-100
        case PK_SUB:    // csg/difference.rs:57-106
        case PK_XFORM:  // tf_facade.rs:41-55
            if constexpr (kOneSite) {
                int wk;
                return composite_t(S, P, r, tmin, tmax, h, wk);
            } else {
                return composite_t_calls(S, P, r, tmin, tmax, h);
            }
        case PK_MEDIUM: {  // the record is cheap; reuse it (rich scene mode only)
            if (!R) return false;
            Hit f;
            if (!hit(S, pi, r, tmin, tmax, f)) return false;
            h.t1 = f.t1; h.t2 = f.t2; h.p = f.p;
            return true;
        }
        }
        return false;
    }

    // CSG and TfFacade decisions through ONE call site of the level below per kind of query: the
    // children are visited by a loop that is not unrolled. Inlining the object switch once per child
    // and per level made the nest-2 extend kernel 397 KB of code, far past the instruction cache.
    // the calls variant (generic / rich mode, where each level below is a real call): one site per
    // child, as a loop around a call would keep its state live across the call (X1 / X2 slower)
    static __device__ __forceinline__ bool composite_t_calls(const DScene& S, const DPrim& P, const Ray& r, double tmin,
                                                             double tmax, HitT& h) {
        switch (P.kind) {
        case PK_AND: {  // csg/intersection.rs:58-100
            const DCsg C = S.csgs[P.idx];
            HitT h1, h2;
            if (!Obj<L - 1, R>::hit_t(S, C.a, r, tmin, tmax, h1)) return false;
            if (!Obj<L - 1, R>::hit_t(S, C.b, r, tmin, tmax, h2)) return false;
            const bool first1 = h1.t1 < h2.t1;
            const int o0 = first1 ? C.a : C.b, o1 = first1 ? C.b : C.a;
            const V3 p0 = first1 ? h1.p : h2.p, p1 = first1 ? h2.p : h1.p;
            if (Obj<L - 1, R>::contains(S, o1, p0)) h = first1 ? h1 : h2;
            else if (Obj<L - 1, R>::contains(S, o0, p1)) h = first1 ? h2 : h1;
            else return false;
            return true;
        }
        case PK_SUB: {  // csg/difference.rs:57-106
            const DCsg C = S.csgs[P.idx];
            HitT hp, hm;
            if (!Obj<L - 1, R>::hit_t(S, C.a, r, tmin, tmax, hp)) return false;
            if (!Obj<L - 1, R>::hit_t(S, C.b, r, tmin, tmax, hm)) { h = hp; return true; }
            if (hp.t1 < hm.t1) {
                if (Obj<L - 1, R>::contains(S, C.b, hp.p)) return false;
                h = hp;
            } else if (hm.t2 < hp.t1) {
                h = hp;
            } else if (hm.t2 < hp.t2) {
                h.p = ray_at(r, hm.t2); h.t1 = hm.t2; h.t2 = hp.t2;
            } else {
                return false;
            }
            return true;
        }
        case PK_XFORM: {  // tf_facade.rs:41-55
            const DXform X = S.xforms[P.idx];
            Ray rr;
            rr.o = r.o; rr.d = r.d;
            tf_inverse_ray(S, X, P.aux, rr.o, rr.d);
            rr.time = r.time;
            if (R) rr.key = r.key;
            if (!Obj<L - 1, R>::hit_t(S, X.child, rr, tmin, tmax, h)) return false;
            h.p = tf_forward(S, X, P.aux, h.p, 1.0);
            return true;
        }
        }
        return false;
    }

    // wk: whose record h is -- 0 the first child (Intersection / Difference: a; TfFacade: its child),
    // 1 the second (b), 2 Difference's synthesized back-face hit of b
    static __device__ __forceinline__ bool composite_t(const DScene& S, const DPrim& P, const Ray& r, double tmin,
                                                       double tmax, HitT& h, int& wk) {
        wk = 0;
        const bool xf = P.kind == PK_XFORM;
        int c0, c1 = -1;
        Ray rr = r;
        DXform X;
        if (xf) {
            X = S.xforms[P.idx];
            c0 = X.child;
            tf_inverse_ray(S, X, P.aux, rr.o, rr.d);
        } else {
            const DCsg C = S.csgs[P.idx];
            c0 = C.a;
            c1 = C.b;
        }
        HitT h1, h2;
        bool ok2 = false;
#pragma clang loop unroll(disable)
        for (int k = 0; k < 2; ++k) {
            HitT t;
            const bool ok = Obj<L - 1, R>::hit_t(S, k ? c1 : c0, rr, tmin, tmax, t);
            if (k == 0) {
                if (!ok) return false;
                h1 = t;
                if (xf) break;
            } else {
                ok2 = ok;
                h2 = t;
            }
        }
        if (xf) {
            h = h1;
            h.p = tf_forward(S, X, P.aux, h1.p, 1.0);
            return true;
        }
        // the contains() queries, first match wins: Intersection asks (o1, p0) then (o0, p1);
        // Difference asks (b, hp.p) when its plus hit comes first
        int q0 = -1, q1 = -1;
        V3 qp0 = h1.p, qp1 = h1.p;
        bool first1 = false;
        if (P.kind == PK_AND) {
            if (!ok2) return false;
            first1 = h1.t1 < h2.t1;
            q0 = first1 ? c1 : c0;       // o1
            q1 = first1 ? c0 : c1;       // o0
            qp0 = first1 ? h1.p : h2.p;  // p0
            qp1 = first1 ? h2.p : h1.p;  // p1
        } else {
            if (!ok2) { h = h1; return true; }
            if (h1.t1 < h2.t1) {
                q0 = c1;
            } else if (h2.t2 < h1.t1) {
                h = h1;
                return true;
            } else if (h2.t2 < h1.t2) {
                // rr is r bit for bit here (not a TfFacade): r itself need not stay live across the
                // children's tests
                h.p = ray_at(rr, h2.t2); h.t1 = h2.t2; h.t2 = h1.t2;
                wk = 2;
                return true;
            } else {
                return false;
            }
        }
        int win = -1;
#pragma clang loop unroll(disable)
        for (int k = 0; k < 2; ++k) {
            const int q = k ? q1 : q0;
            if (q < 0) break;
            if (Obj<L - 1, R>::contains(S, q, k ? qp1 : qp0)) { win = k; break; }
        }
        if (P.kind == PK_AND) {
            if (win < 0) return false;
            wk = ((win == 0) == first1) ? 0 : 1;  // (o1 contains p0): the first hit, else the second
            h = wk == 0 ? h1 : h2;
            return true;
        }
        if (win >= 0) return false;  // Difference: the plus hit lies inside the minus object
        h = h1;
        return true;
    }

    static __device__ __forceinline__ bool composite_hit_calls(const DScene& S, const DPrim& P, const Ray& r, double tmin,
                                                               double tmax, Hit& h) {
        switch (P.kind) {
        case PK_AND: {  // csg/intersection.rs:58-100: decided on (t1, t2, p), then the winner's record
            const DCsg C = S.csgs[P.idx];
            HitT h1, h2;
            if (!Obj<L - 1, R>::hit_t(S, C.a, r, tmin, tmax, h1)) return false;
            if (!Obj<L - 1, R>::hit_t(S, C.b, r, tmin, tmax, h2)) return false;
            const bool first1 = h1.t1 < h2.t1;
            const int o0 = first1 ? C.a : C.b, o1 = first1 ? C.b : C.a;
            const V3 p0 = first1 ? h1.p : h2.p, p1 = first1 ? h2.p : h1.p;
            int win;
            if (Obj<L - 1, R>::contains(S, o1, p0)) win = o0;
            else if (Obj<L - 1, R>::contains(S, o0, p1)) win = o1;
            else return false;
            Obj<L - 1, R>::hit(S, win, r, tmin, tmax, h);
            if (h.mat < 0) h.mat = P.mat;  // set_material_if_none (hit.rs:69-78)
            return true;
        }
        case PK_SUB: {  // csg/difference.rs:57-106
            const DCsg C = S.csgs[P.idx];
            HitT hp, hm;
            if (!Obj<L - 1, R>::hit_t(S, C.a, r, tmin, tmax, hp)) return false;
            bool plus;
            if (!Obj<L - 1, R>::hit_t(S, C.b, r, tmin, tmax, hm)) plus = true;
            else if (hp.t1 < hm.t1) {
                if (Obj<L - 1, R>::contains(S, C.b, hp.p)) return false;
                plus = true;
            } else plus = hm.t2 < hp.t1;
            if (plus) {
                Obj<L - 1, R>::hit(S, C.a, r, tmin, tmax, h);
            } else if (hm.t2 < hp.t2) {
                V3 p = ray_at(r, hm.t2);
                V3 n = shape_normal(S, C.b, p);
                h.p = p; h.n = -n; h.mat = S.prims[C.b].mat; h.t1 = hm.t2; h.t2 = hp.t2; h.outside = 1;
                if (R) { h.u = 0.0; h.v = 0.0; }
            } else {
                return false;
            }
            if (h.mat < 0) h.mat = P.mat;
            return true;
        }
        case PK_XFORM: {  // tf_facade.rs:41-55 (normal stays in object space, t unchanged)
            const DXform X = S.xforms[P.idx];
            Ray rr;
            rr.o = r.o; rr.d = r.d;
            tf_inverse_ray(S, X, P.aux, rr.o, rr.d);
            rr.time = r.time;
            if (R) rr.key = r.key;
            if (!Obj<L - 1, R>::hit(S, X.child, rr, tmin, tmax, h)) return false;
            h.p = tf_forward(S, X, P.aux, h.p, 1.0);
            return true;
        }
        }
        return false;
    }

    static __device__ bool hit(const DScene& S, int pi, const Ray& r, double tmin, double tmax, Hit& h) {
        const DPrim P = S.prims[pi];
        switch (P.kind) {
        case PK_SPHERE: return sphere_hit(S.spheres[P.idx], P.mat, r, tmin, tmax, h, R ? S.uv : 0);
        case PK_RECT: {
            const DRect& Q = S.rects[P.idx];
            return rect_hit_raw(Q.ax0, Q.ax1, Q.ax2, Q.k, Q.a0, Q.a1, Q.b0, Q.b1, P.mat, r, tmin, tmax, h, R ? S.uv : 0);
        }
        case PK_BOX: return box_hit(S.boxes[P.idx], P.mat, r, tmin, tmax, h, R ? S.uv : 0);
        case PK_QUADRIC: return quadric_hit(S.quadrics[P.idx], P.mat, r, tmin, tmax, h, R ? S.uv : 0);
        case PK_TRIANGLE: return tri_hit(S.tris[P.idx], P.mat, r, tmin, tmax, h, R ? S.uv : 0);
        case PK_AND:      // csg/intersection.rs:58-100: decided on (t1, t2, p), then the winner's record
        case PK_SUB:      // csg/difference.rs:57-106
        case PK_XFORM: {  // tf_facade.rs:41-55 (normal stays in object space, t unchanged)
            if constexpr (!kOneSite) return composite_hit_calls(S, P, r, tmin, tmax, h);
            const bool xf = P.kind == PK_XFORM;
            int child;
            Ray rr = r;
            DXform X;
            if (xf) {
                X = S.xforms[P.idx];
                child = X.child;
                rr.o = r.o; rr.d = r.d;
                tf_inverse_ray(S, X, P.aux, rr.o, rr.d);
            } else {
                HitT t;
                int wk;
                if (!composite_t(S, P, r, tmin, tmax, t, wk)) return false;
                const DCsg C = S.csgs[P.idx];
                if (wk == 2) {  // Difference: the minus object's far hit, facing out of the plus one
                    const V3 n = shape_normal(S, C.b, t.p);
                    h.p = t.p; h.n = -n; h.mat = S.prims[C.b].mat; h.t1 = t.t1; h.t2 = t.t2; h.outside = 1;
                    if (R) { h.u = 0.0; h.v = 0.0; }
                    if (h.mat < 0) h.mat = P.mat;
                    return true;
                }
                child = wk ? C.b : C.a;
            }
            // the winner's own record (one call site of the level below)
            const bool ok = Obj<L - 1, R>::hit(S, child, rr, tmin, tmax, h);
            if (xf) {
                if (!ok) return false;
                h.p = tf_forward(S, X, P.aux, h.p, 1.0);
                return true;
            }
            if (h.mat < 0) h.mat = P.mat;  // set_material_if_none (hit.rs:69-78)
            return true;
        }
        case PK_MEDIUM: {  // medium/constant.rs:42-84
            if (!R) return false;  // media exist only in the rich scene mode
            const DMedium M = S.media[P.idx];
            // the boundary's two hits decide on their t1 alone: hit_t (the same t1 bit for bit, no record: a
            // sphere boundary's (u, v) -- correctly rounded atan2 / asin in image-textured scenes -- is never read)
            HitT h1, h2;
            if (!Obj<L - 1, R>::hit_t(S, M.boundary, r, -RS_INF, RS_INF, h1)) return false;
            if (!Obj<L - 1, R>::hit_t(S, M.boundary, r, h1.t1 + 0.0001, RS_INF, h2)) return false;
            double t1 = h1.t1, t2 = h2.t1;
            if (t1 < tmin) t1 = tmin;
            if (t2 > tmax) t2 = tmax;
            if (t1 >= t2) return false;
            if (t1 < 0.0) t1 = 0.0;
            const double length_per_unit = sqrt(len2(r.d));
            const double distance_inside = (t2 - t1) * length_per_unit;
            const double hit_distance = M.neg_inv_density * rs_cr::log_cr(medium_uniform(r.key, pi));
            if (hit_distance > distance_inside) return false;
            const double th = t1 + hit_distance / length_per_unit;
            h.p = ray_at(r, th);
            h.n = v3(1.0, 0.0, 0.0);
            h.mat = M.mat; h.t1 = th; h.t2 = th; h.u = 0.0; h.v = 0.0; h.outside = 0;
            return true;
        }
        }
        return false;
    }

    static __device__ __forceinline__ bool contains(const DScene& S, int pi, V3 p) {
        if constexpr (L <= 2 && R == 0) return contains_body(S, pi, p);
        else return contains_call(S, pi, p);
    }
    static __device__ __noinline__ bool contains_call(const DScene& S, int pi, V3 p) { return contains_body(S, pi, p); }
    static __device__ __forceinline__ bool contains_calls(const DScene& S, const DPrim& P, V3 p) {
        switch (P.kind) {
        case PK_AND: { const DCsg C = S.csgs[P.idx]; return Obj<L - 1, R>::contains(S, C.a, p) && Obj<L - 1, R>::contains(S, C.b, p); }
        case PK_SUB: { const DCsg C = S.csgs[P.idx]; return Obj<L - 1, R>::contains(S, C.a, p) && !Obj<L - 1, R>::contains(S, C.b, p); }
        case PK_XFORM: {
            const DXform X = S.xforms[P.idx];
            return Obj<L - 1, R>::contains(S, X.child, tf_inverse(S, X, P.aux, p, 1.0));
        }
        default: return false;
        }
    }
    static __device__ __forceinline__ bool contains_body(const DScene& S, int pi, V3 p) {
        const DPrim P = S.prims[pi];
        switch (P.kind) {
        case PK_SPHERE: {  // sphere.rs:111-115
            const DSphere& s = S.spheres[P.idx];
            V3 d = ld3(s.c) - p;
            return len2(d) < s.r * s.r;
        }
        case PK_BOX: return box_contains(S.boxes[P.idx], p);
        case PK_QUADRIC: return quadric_contains(S.quadrics[P.idx], p);
        case PK_AND:    // a && b
        case PK_SUB:    // a && !b
        case PK_XFORM: {  // child at the inverse-transformed point
            // one call site of the level below (loop not unrolled), as in composite_t
            if constexpr (!kOneSite) return contains_calls(S, P, p);
            const bool xf = P.kind == PK_XFORM;
            int c0, c1 = -1;
            V3 q = p;
            if (xf) {
                const DXform X = S.xforms[P.idx];
                c0 = X.child;
                q = tf_inverse(S, X, P.aux, p, 1.0);
            } else {
                const DCsg C = S.csgs[P.idx];
                c0 = C.a;
                c1 = C.b;
            }
#pragma clang loop unroll(disable)
            for (int k = 0; k < 2; ++k) {
                const bool in = Obj<L - 1, R>::contains(S, k ? c1 : c0, q);
                if (k == 0) {
                    if (xf) return in;
                    if (!in) return false;
                } else {
                    return P.kind == PK_AND ? in : !in;
                }
            }
            return false;
        }
        default: return false;  // AARect / Triangle: false; ConstantMedium: unimplemented! upstream (constant.rs:86-91)
        }
    }

    // Hittable::random of a light (only called for objects in the lights list)
    static __device__ V3 random(const DScene& S, int pi, V3 origin, Rng& rng) {
        const DPrim P = S.prims[pi];
        switch (P.kind) {
        case PK_SPHERE: return sphere_random(S.spheres[P.idx], origin, rng);
        case PK_RECT: {  // rect.rs:141-153 (xz only upstream; returns origin - point)
            const DRect& Q = S.rects[P.idx];
            V3 root = v3(0.0, Q.k, 0.0);
            root.x = rng.range(Q.a0, Q.a1);
            root.z = rng.range(Q.b0, Q.b1);
            return origin - root;
        }
        case PK_QUADRIC: return -origin;                                   // quadric.rs:202-205
        case PK_TRIANGLE: return origin - ld3(S.tris[P.idx].p0);          // triangle_mesh.rs:137-139
        case PK_AND: return Obj<L - 1, R>::random(S, S.csgs[P.idx].a, origin, rng);
        case PK_SUB: return Obj<L - 1, R>::random(S, S.csgs[P.idx].a, origin, rng);
        case PK_XFORM: {
            const DXform X = S.xforms[P.idx];
            return Obj<L - 1, R>::random(S, X.child, tf_inverse(S, X, P.aux, origin, 1.0), rng);
        }
        default: return v3(1.0, 0.0, 0.0);  // Box / BVH / ConstantMedium (constant.rs:97-99)
        }
    }

    static __device__ V3 shape_normal(const DScene& S, int pi, V3 p) {
        const DPrim P = S.prims[pi];
        switch (P.kind) {
        case PK_SPHERE: return sphere_normal(S.spheres[P.idx], p);
        case PK_RECT: { int a = S.rects[P.idx].ax2; return v3(a == 0, a == 1, a == 2); }
        case PK_QUADRIC: return quadric_normal(S.quadrics[P.idx], p);
        default: return v3(0.0, 1.0, 0.0);  // Box::normal (box.rs:114-116)
        }
    }

    // ONB::build_from (onb.rs:26-40) + Sphere::random (sphere.rs:149-164): radius ignored
    static __device__ V3 sphere_random(const DSphere& s, V3 origin, Rng& rng);
};

// ------------------------------------------------------------------ ONB / PDFs ----
struct Onb { V3 u, v, w; };
__device__ __forceinline__ Onb onb_from(V3 n) {
    Onb o;
    o.w = unit(n);
    V3 uc = cross(v3(0.0, 1.0, 0.0), o.w);
    o.u = len2(uc) < 0.00000001 ? unit(cross(v3(1.0, 0.0, 0.0), o.w)) : unit(uc);
    o.v = cross(o.w, o.u);
    return o;
}
__device__ __forceinline__ V3 onb_local(const Onb& o, V3 a) {  // onb.rs:14-24
    return v3(o.u.x * a.x + o.v.x * a.y + o.w.x * a.z, o.u.y * a.x + o.v.y * a.y + o.w.y * a.z,
              o.u.z * a.x + o.v.z * a.y + o.w.z * a.z);
}

template <int L, int R>
__device__ V3 Obj<L, R>::sphere_random(const DSphere& s, V3 origin, Rng& rng) {
    V3 c = ld3(s.c);
    Onb uvw = onb_from(c - origin);
    for (int i = 0; i < RS_REJECTION_CAP; ++i) {
        V3 u = uvw.u * rng.gen();
        V3 v = uvw.v * rng.gen();
        V3 uv = u + v;
        if (len2(uv) < 1.0) return (uv + c) - origin;
    }
    return c - origin;
}

// vec3.rs:100-111
__device__ __forceinline__ V3 random_cosine_direction(Rng& rng) {
    double r1 = rng.gen();
    double r2 = rng.gen();
    double q2 = sqrt(r2);
    double phi = 2.0 * RS_PI * r1;
    double sp, cp;
    rs_cr::sincos_cr(phi, &sp, &cp);  // correctly rounded (rs_crmath.h)
    return v3(cp * q2, sp * q2, sqrt(1.0 - r2));
}
// vec3.rs:115-126
__device__ __forceinline__ V3 random_cosine_direction_exponent(double e, Rng& rng) {
    double r1 = rng.gen();
    double r2 = rs_cr::pow_cr(rng.gen(), 1.0 / (e + 1.0));
    double st = sqrt(1.0 - r2 * r2);
    double phi = 2.0 * RS_PI * r1;
    double sp, cp;
    rs_cr::sincos_cr(phi, &sp, &cp);
    return v3(cp * st, sp * st, r2);
}

// vec3.rs:91-96
__device__ __forceinline__ V3 random_unit(Rng& rng) {
    const double a = rng.range(0.0, 2.0 * RS_PI);
    const double z = rng.range(-1.0, 1.0);
    const double r = sqrt(1.0 - z * z);
    double sa, ca;
    rs_cr::sincos_cr(a, &sa, &ca);
    return v3(r * ca, r * sa, z);
}

// CosinePdf (pdf.rs:20-49) / ReflectionPdf (pdf.rs:86-141) / SpherePdf (pdf.rs:215-238) /
// BlinnPhongPdf (pdf.rs:144-212)
enum PdfKind { kPdfCosine = 0, kPdfReflection = 1, kPdfSphere = 2, kPdfBlinnPhong = 3 };
struct Pdf {
    int kind;      // PdfKind
    Onb n;         // cosine: about normal; reflection / Blinn-Phong: onb_normal
    Onb refl;      // reflection / Blinn-Phong: onb_reflected
    double exponent;
    V3 rin;        // Blinn-Phong: r_in_direction
    double k;      // Blinn-Phong: k_specular
};
// the Phong lobe about onb_reflected, rejected until it leaves the surface (pdf.rs:118-134, :196-206)
__device__ __forceinline__ V3 phong_lobe(const Pdf& p, Rng& rng) {
    for (int i = 0; i < RS_REJECTION_CAP; ++i) {
        V3 d = onb_local(p.refl, random_cosine_direction_exponent(p.exponent, rng));
        if (dot(d, p.n.w) > 0.0) return d;
    }
    return p.n.w;
}
// R = 0: only the cosine and reflection PDFs exist (Isotropic / BlinnPhong are rich-mode materials)
template <int R>
__device__ __forceinline__ double pdf_value(const Pdf& p, V3 d) {
    if (p.kind == kPdfCosine) { double c = dot(d, p.n.w); return c < 0.0 ? 0.0 : c / RS_PI; }
    if (R && p.kind == kPdfSphere) return 1.0 / (4.0 * RS_PI);
    if (R && p.kind == kPdfBlinnPhong) {  // pdf.rs:177-193
        const double cosine = dot(d, p.n.w);
        const V3 random_normal = unit(-p.rin + d);
        const double cosine_specular = fmax(dot(random_normal, p.n.w), 0.0);
        const double normal_pdf = (p.exponent + 1.0) / (2.0 * RS_PI) * rs_cr::pow_cr(cosine_specular, p.exponent);
        return fmax(cosine / RS_PI, 0.0) * (1.0 - p.k) + normal_pdf / (4.0 * dot(p.rin * -1.0, random_normal)) * p.k;
    }
    double v = dot(d, p.refl.w) / RS_PI;
    return v < 0.0 ? 0.0 : v;
}
template <int R>
__device__ __forceinline__ V3 pdf_generate(const Pdf& p, Rng& rng) {
    if (p.kind == kPdfCosine) return onb_local(p.n, random_cosine_direction(rng));
    if (R && p.kind == kPdfSphere) return random_unit(rng);
    if (R && p.kind == kPdfBlinnPhong) {  // pdf.rs:196-211
        if (rng.gen() < p.k) return phong_lobe(p, rng);
        return onb_local(p.n, random_cosine_direction(rng));
    }
    return phong_lobe(p, rng);
}

// ------------------------------------------------------------------ textures ----
// Rust `as isize` / `as u32` from f64: truncation toward zero, saturating, NaN -> 0
__device__ __forceinline__ int64_t as_isize(double x) {
    if (!(x == x)) return 0;
    if (x >= 9223372036854775807.0) return INT64_MAX;
    if (x <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)x;
}
__device__ __forceinline__ uint32_t as_u32(double x) {
    if (!(x > 0.0)) return 0u;
    if (x >= 4294967295.0) return 0xffffffffu;
    return (uint32_t)x;
}

// Perlin::noise (noise.rs:111-148) + interpolate (:170-207). Sums start from 0.0 (f64 Sum).
__device__ double perlin_noise(const DScene& S, const DPerlin& P, V3 p) {
    const int64_t mask = (int64_t)P.point_count - 1;
    const double* val = S.tex_f64 + P.voff;
    const int32_t* px = S.tex_i32 + P.poff;
    const int32_t* py = px + P.point_count;
    const int32_t* pz = py + P.point_count;
    if (P.smooth == RS_SMOOTH_NONE) {
        const int64_t i = as_isize(4.0 * p.x) & mask, j = as_isize(4.0 * p.y) & mask, k = as_isize(4.0 * p.z) & mask;
        const int idx = px[i] ^ py[j] ^ pz[k];
        return P.vector ? val[3 * idx] : val[idx];
    }
    const int64_t i = as_isize(floor(p.x)), j = as_isize(floor(p.y)), k = as_isize(floor(p.z));
    const double u = p.x - (double)i, v = p.y - (double)j, w = p.z - (double)k;
    double uu = u, vv = v, ww = w;
    if (P.smooth == RS_SMOOTH_HERMITE) {
        uu = u * u * (3.0 - 2.0 * u);
        vv = v * v * (3.0 - 2.0 * v);
        ww = w * w * (3.0 - 2.0 * w);
    }
    double si = 0.0;
    for (int di = 0; di < 2; ++di) {
        double sj = 0.0;
        for (int dj = 0; dj < 2; ++dj) {
            double sk = 0.0;
            for (int dk = 0; dk < 2; ++dk) {
                const int64_t xi = (int64_t)((uint64_t)i + (uint64_t)di) & mask;  // wrapping add
                const int64_t yi = (int64_t)((uint64_t)j + (uint64_t)dj) & mask;
                const int64_t zi = (int64_t)((uint64_t)k + (uint64_t)dk) & mask;
                const int idx = px[xi] ^ py[yi] ^ pz[zi];
                double c;
                if (P.vector) {
                    const V3 weight = v3(u - (double)di, v - (double)dj, w - (double)dk);
                    c = dot(ld3(val + 3 * idx), weight);
                } else {
                    c = val[idx];
                }
                sk = sk + fma((double)di, uu, (double)(1 - di) * (1.0 - uu)) *
                              fma((double)dj, vv, (double)(1 - dj) * (1.0 - vv)) *
                              fma((double)dk, ww, (double)(1 - dk) * (1.0 - ww)) * c;
            }
            sj = sj + sk;
        }
        si = si + sj;
    }
    return si;
}
// Perlin::calculate_turbulence (noise.rs:150-166)
__device__ double perlin_turbulence(const DScene& S, const DPerlin& P, V3 p, int depth) {
    double weight = 1.0, acc = 0.0;
    for (int d = 0; d < depth; ++d) {
        acc = acc + weight * perlin_noise(S, P, p);
        weight *= 0.5;
        p = v3(p.x * 2.0, p.y * 2.0, p.z * 2.0);
    }
    return fabs(acc);
}
// Perlin as a Texture (noise.rs:187-211): Color(1,1,1,1) * value (Color * f64 = channel * value as f32)
__device__ __noinline__ double perlin_value(const DScene& S, const DPerlin& P, V3 point) {
    if (P.type == RS_PERLIN_TURBULENCE) return perlin_turbulence(S, P, point, P.depth);
    if (P.type == RS_PERLIN_MARBLE) {
        const double noise = perlin_turbulence(S, P, point, P.depth);
        return (rs_cr::sin_cr(fma(P.scale, point.z, 10.0 * noise)) + 1.0) * 0.5;
    }
    double noise = perlin_noise(S, P, v3(P.scale * point.x, P.scale * point.y, P.scale * point.z));
    if (P.vector) noise = 0.5 * (noise + 1.0);
    return noise;
}

// Image::color (image.rs:34-50) as packed 8-bit rgb (out of line, like perlin_value)
__device__ __noinline__ uint32_t image_texel(const DScene& S, int id, double u, double v) {
    const DImage I = S.images[id];
    const double vv = 1.0 - v;
    uint32_t x = as_u32(u * (double)I.w), y = as_u32(vv * (double)I.h);
    if (x >= I.w) x = I.w - 1;
    if (y >= I.h) y = I.h - 1;
    const uint8_t* px = S.tex_u8 + I.off + 3 * ((uint64_t)y * I.w + x);
    return (uint32_t)px[0] | ((uint32_t)px[1] << 8) | ((uint32_t)px[2] << 16);
}

// texture eval: Color (color.rs:61-65) / Checker (checker.rs:21-30) / Perlin / Image (image.rs:34-50);
// R = 0 (every scene mode but the rich one) compiles Color / Checker only
template <int R>
__device__ __forceinline__ void tex_color(const DScene& S, const DMaterial& m, V3 p, double u, double v, float c[3]) {
    if (R && m.tex_kind == RS_TEX_PERLIN) {
        const float f = (float)perlin_value(S, S.perlins[m.tex_data], p);
        c[0] = 1.0f * f; c[1] = 1.0f * f; c[2] = 1.0f * f;
        return;
    }
    if (R && m.tex_kind == RS_TEX_IMAGE) {
        const uint32_t t = image_texel(S, m.tex_data, u, v);
        c[0] = (float)(t & 255u) / 255.0f; c[1] = (float)((t >> 8) & 255u) / 255.0f; c[2] = (float)(t >> 16) / 255.0f;
        return;
    }
    bool odd = false;
    if (m.tex_kind == RS_TEX_CHECKER) {
        odd = rs_cr::sin3_negative(m.tex_scale * p.x, m.tex_scale * p.y, m.tex_scale * p.z);
    }
    const float* s = odd ? m.odd : m.even;
    c[0] = s[0]; c[1] = s[1]; c[2] = s[2];
}
template <int R>
__device__ __forceinline__ void tex_color(const DScene& S, const DMaterial& m, const Hit& h, float c[3]) {
    tex_color<R>(S, m, h.p, h.u, h.v, c);
}

// ------------------------------------------------------------------ materials ----

// compiler-rt __powidf2 (phong powi with a runtime exponent)
__device__ __forceinline__ double powi_rt(double a, int b) {
    const int recip = b < 0;
    double r = 1;
    while (1) {
        if (b & 1) r *= a;
        b /= 2;
        if (b == 0) break;
        a *= a;
    }
    return recip ? 1 / r : r;
}

// color.rs:50-58 (f32 gradient), t = (d.y + 1) * 0.5 (rtow_13_1.rs:38-41)
__device__ __forceinline__ V3 background(const DScene& S, const Ray& r) {
    double t = (r.d.y + 1.0) * 0.5;
    float a = (float)fmin(fmax(t, 0.0), 1.0);
    float b = 1.0f - a;
    float cr = S.bg_lo[0] * b + S.bg_hi[0] * a;
    float cg = S.bg_lo[1] * b + S.bg_hi[1] * a;
    float cb = S.bg_lo[2] * b + S.bg_hi[2] * a;
    return v3((double)cr, (double)cg, (double)cb);
}

// camera.rs:77-85 + vec3.rs:140-147
__device__ __forceinline__ Ray camera_ray(const DCamera& c, double u, double v, Rng& rng) {
    V3 disk = v3(0.0, 0.0, 0.0);
    for (int i = 0; i < RS_REJECTION_CAP; ++i) {
        double px = rng.range(-1.0, 1.0);
        double py = rng.range(-1.0, 1.0);
        V3 p = v3(px, py, 0.0);
        if (len2(p) < 1.0) { disk = p; break; }
    }
    V3 rd = (c.aperture / 2.0) * disk;
    V3 offset = ld3(c.hu) * rd.x + ld3(c.vu) * rd.y;
    V3 o = ld3(c.origin) + offset;
    V3 dir = ld3(c.lb) + u * ld3(c.hf) + v * ld3(c.vf) - o;
    Ray r;
    r.o = o;
    r.d = unit(dir);
    r.time = c.shutter * rng.gen();
    r.key = 0;
    return r;
}

}  // namespace rs
