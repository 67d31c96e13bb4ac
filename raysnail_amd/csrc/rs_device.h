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

struct Ray { V3 o, d; double time; };
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
};

// ------------------------------------------------------------------ hit record ----
struct Hit {
    V3 p, n;
    double t1, t2;
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

__device__ __forceinline__ bool sphere_hit(const DSphere& s, int32_t mat, const Ray& r, double tmin, double tmax, Hit& h) {
    double t, t2;
    if (!sphere_t(s, r, tmin, tmax, t, t2)) return false;
    V3 p = ray_at(r, t);
    finish_rec(h, r, t, t2, sphere_normal(s, p), mat);
    return true;
}

// rect.rs:101-120
__device__ __forceinline__ bool rect_hit_raw(int ax0, int ax1, int ax2, double k, double a0, double a1, double b0, double b1,
                                             int32_t mat, const Ray& r, double tmin, double tmax, Hit& h) {
    double t1 = (k - comp(r.o, ax2)) / comp(r.d, ax2);
    if (!in_range(t1, tmin, tmax)) return false;
    double a = fma(t1, comp(r.d, ax0), comp(r.o, ax0));
    if (a < a0 || a > a1) return false;
    double b = fma(t1, comp(r.d, ax1), comp(r.o, ax1));
    if (b < b0 || b > b1) return false;
    V3 n = v3(ax2 == 0 ? 1.0 : 0.0, ax2 == 1 ? 1.0 : 0.0, ax2 == 2 ? 1.0 : 0.0);
    finish_rec(h, r, t1, RS_FMAX, n, mat);
    return true;
}

// box.rs:125-149; faces in the order built by box.rs:55-105
__device__ bool box_hit(const DBox& b, int32_t mat, const Ray& r, double tmin, double tmax, Hit& h) {
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
            if (rect_hit_raw(ax0, ax1, ax2, k, a0, a1, b0, b1, mat, r, tmin, tmax, t)) {
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
// quadric.rs:112-182
__device__ bool quadric_hit(const DQuadric& Q, int32_t mat, const Ray& r, double tmin, double tmax, Hit& h) {
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
    return true;
}
__device__ __forceinline__ bool quadric_contains(const DQuadric& Q, V3 p) {  // quadric.rs:184-189
    const double* q = Q.q;
    return (p.x * (q[0] * p.x + q[1] * p.y + q[3]) + p.y * (q[4] * p.y + q[5] * p.z + q[6]) +
            p.z * (q[7] * p.z + q[2] * p.x + q[8]) + q[9]) <= 0.0;
}

// triangle_mesh.rs:85-131
// tri_hit's accept test alone (the traversal's leaf test; the winner's record is recomputed)
__device__ __forceinline__ bool tri_t(const DTri& T, const Ray& r, double tmin, double tmax, double& t_out) {
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
    t_out = t;
    return true;
}

__device__ bool tri_hit(const DTri& T, int32_t mat, const Ray& r, double tmin, double tmax, Hit& h) {
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

// ------------------------------------------------------------------ objects (nested) ----
template <int L> struct Obj;

template <> struct Obj<-1> {
    static __device__ bool hit(const DScene&, int, const Ray&, double, double, Hit&) { return false; }
    static __device__ bool contains(const DScene&, int, V3) { return false; }
    static __device__ V3 random(const DScene&, int, V3, Rng&) { return v3(1.0, 0.0, 0.0); }
};

template <int L> struct Obj {
    static __device__ bool hit(const DScene& S, int pi, const Ray& r, double tmin, double tmax, Hit& h) {
        const DPrim P = S.prims[pi];
        switch (P.kind) {
        case PK_SPHERE: return sphere_hit(S.spheres[P.idx], P.mat, r, tmin, tmax, h);
        case PK_RECT: {
            const DRect& R = S.rects[P.idx];
            return rect_hit_raw(R.ax0, R.ax1, R.ax2, R.k, R.a0, R.a1, R.b0, R.b1, P.mat, r, tmin, tmax, h);
        }
        case PK_BOX: return box_hit(S.boxes[P.idx], P.mat, r, tmin, tmax, h);
        case PK_QUADRIC: return quadric_hit(S.quadrics[P.idx], P.mat, r, tmin, tmax, h);
        case PK_TRIANGLE: return tri_hit(S.tris[P.idx], P.mat, r, tmin, tmax, h);
        case PK_AND: {  // csg/intersection.rs:58-100
            const DCsg C = S.csgs[P.idx];
            Hit h1, h2;
            bool ok1 = Obj<L - 1>::hit(S, C.a, r, tmin, tmax, h1);
            bool ok2 = Obj<L - 1>::hit(S, C.b, r, tmin, tmax, h2);
            if (!(ok1 && ok2)) return false;
            const bool first1 = h1.t1 < h2.t1;
            const int o0 = first1 ? C.a : C.b, o1 = first1 ? C.b : C.a;
            const V3 p0 = first1 ? h1.p : h2.p, p1 = first1 ? h2.p : h1.p;
            if (Obj<L - 1>::contains(S, o1, p0)) { h = first1 ? h1 : h2; }
            else if (Obj<L - 1>::contains(S, o0, p1)) { h = first1 ? h2 : h1; }
            else return false;
            if (h.mat < 0) h.mat = P.mat;  // set_material_if_none (hit.rs:69-78)
            return true;
        }
        case PK_SUB: {  // csg/difference.rs:57-106
            const DCsg C = S.csgs[P.idx];
            Hit hp, hm;
            bool okp = Obj<L - 1>::hit(S, C.a, r, tmin, tmax, hp);
            bool okm = Obj<L - 1>::hit(S, C.b, r, tmin, tmax, hm);
            if (!okp) return false;
            if (!okm) { h = hp; return true; }
            if (hp.t1 < hm.t1) {
                if (Obj<L - 1>::contains(S, C.b, hp.p)) return false;
                h = hp;
            } else if (hm.t2 < hp.t1) {
                h = hp;
            } else if (hm.t2 < hp.t2) {
                V3 p = ray_at(r, hm.t2);
                V3 n = shape_normal(S, C.b, p);
                h.p = p; h.n = -n; h.mat = S.prims[C.b].mat; h.t1 = hm.t2; h.t2 = hp.t2; h.outside = 1;
            } else {
                return false;
            }
            if (h.mat < 0) h.mat = P.mat;
            return true;
        }
        case PK_XFORM: {  // tf_facade.rs:41-55 (normal stays in object space, t unchanged)
            const DXform X = S.xforms[P.idx];
            Ray rr;
            rr.o = tf_inverse(S, X, P.aux, r.o, 1.0);
            rr.d = tf_inverse(S, X, P.aux, r.d, 0.0);
            rr.time = r.time;
            if (!Obj<L - 1>::hit(S, X.child, rr, tmin, tmax, h)) return false;
            h.p = tf_forward(S, X, P.aux, h.p, 1.0);
            return true;
        }
        }
        return false;
    }

    static __device__ bool contains(const DScene& S, int pi, V3 p) {
        const DPrim P = S.prims[pi];
        switch (P.kind) {
        case PK_SPHERE: {  // sphere.rs:111-115
            const DSphere& s = S.spheres[P.idx];
            V3 d = ld3(s.c) - p;
            return len2(d) < s.r * s.r;
        }
        case PK_BOX: return box_contains(S.boxes[P.idx], p);
        case PK_QUADRIC: return quadric_contains(S.quadrics[P.idx], p);
        case PK_AND: { const DCsg C = S.csgs[P.idx]; return Obj<L - 1>::contains(S, C.a, p) && Obj<L - 1>::contains(S, C.b, p); }
        case PK_SUB: { const DCsg C = S.csgs[P.idx]; return Obj<L - 1>::contains(S, C.a, p) && !Obj<L - 1>::contains(S, C.b, p); }
        case PK_XFORM: {
            const DXform X = S.xforms[P.idx];
            return Obj<L - 1>::contains(S, X.child, tf_inverse(S, X, P.aux, p, 1.0));
        }
        default: return false;  // AARect / Triangle: false
        }
    }

    // Hittable::random of a light (only called for objects in the lights list)
    static __device__ V3 random(const DScene& S, int pi, V3 origin, Rng& rng) {
        const DPrim P = S.prims[pi];
        switch (P.kind) {
        case PK_SPHERE: return sphere_random(S.spheres[P.idx], origin, rng);
        case PK_RECT: {  // rect.rs:141-153 (xz only upstream; returns origin - point)
            const DRect& R = S.rects[P.idx];
            V3 root = v3(0.0, R.k, 0.0);
            root.x = rng.range(R.a0, R.a1);
            root.z = rng.range(R.b0, R.b1);
            return origin - root;
        }
        case PK_QUADRIC: return -origin;                                   // quadric.rs:202-205
        case PK_TRIANGLE: return origin - ld3(S.tris[P.idx].p0);          // triangle_mesh.rs:137-139
        case PK_AND: return Obj<L - 1>::random(S, S.csgs[P.idx].a, origin, rng);
        case PK_SUB: return Obj<L - 1>::random(S, S.csgs[P.idx].a, origin, rng);
        case PK_XFORM: {
            const DXform X = S.xforms[P.idx];
            return Obj<L - 1>::random(S, X.child, tf_inverse(S, X, P.aux, origin, 1.0), rng);
        }
        default: return v3(1.0, 0.0, 0.0);  // Box / BVH
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

template <int L>
__device__ V3 Obj<L>::sphere_random(const DSphere& s, V3 origin, Rng& rng) {
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

// CosinePdf (pdf.rs:20-49) / ReflectionPdf (pdf.rs:86-141)
struct Pdf {
    int kind;      // 0 cosine, 1 reflection
    Onb n;         // cosine: about normal; reflection: onb_normal
    Onb refl;      // reflection: onb_reflected
    double exponent;
};
__device__ __forceinline__ double pdf_value(const Pdf& p, V3 d) {
    if (p.kind == 0) { double c = dot(d, p.n.w); return c < 0.0 ? 0.0 : c / RS_PI; }
    double v = dot(d, p.refl.w) / RS_PI;
    return v < 0.0 ? 0.0 : v;
}
__device__ __forceinline__ V3 pdf_generate(const Pdf& p, Rng& rng) {
    if (p.kind == 0) return onb_local(p.n, random_cosine_direction(rng));
    for (int i = 0; i < RS_REJECTION_CAP; ++i) {
        V3 d = onb_local(p.refl, random_cosine_direction_exponent(p.exponent, rng));
        if (dot(d, p.n.w) > 0.0) return d;
    }
    return p.n.w;
}

// ------------------------------------------------------------------ materials ----
// texture eval: Color (color.rs:61-65) / Checker (checker.rs:21-30)
__device__ __forceinline__ void tex_color(const DMaterial& m, V3 p, float c[3]) {
    bool odd = false;
    if (m.tex_kind == RS_TEX_CHECKER) {
        odd = rs_cr::sin3_negative(m.tex_scale * p.x, m.tex_scale * p.y, m.tex_scale * p.z);
    }
    const float* s = odd ? m.odd : m.even;
    c[0] = s[0]; c[1] = s[1]; c[2] = s[2];
}

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
    return r;
}

}  // namespace rs
