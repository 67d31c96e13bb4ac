// rs_kernels.hip — gfx950 kernels of the render path.
//
//   k_path_mega   painter.rs:154-187 (render_pixel, one sample) -> camera.rs:77-85 (Camera::ray)
//                 -> camera.rs:156-255 (ray_color, iterated) with BVH traversal (bvh.rs:173-192)
//   k_wfs_extend / k_wfs_shade_all / k_wf_*   the wavefront form of the same recursion
//   k_accumulate  painter.rs:167-179 color_vec sum, in sample order; its last batch also does
//                 vec3.rs:227-240 into_color (/N, sqrt gamma, f32, alpha 1) + painter.rs:204-210 mask
//   k_finalize    into_color alone (frames without samples)
//
// Build with -ffp-contract=off (see Makefile): the f64 arithmetic mirrors the reference's
// operation order (explicit fma() only where raysnail calls mul_add); sin/cos/pow are the
// correctly rounded ones of include/rs_crmath.h on both sides, so GPU frames equal the CPU
// oracle's bit for bit.
#include <cstdlib>

#include <hip/hip_ext.h>

#include "rs_device.h"
#include "rs_internal.h"

// Translation units (Makefile): the scene-mode templates of the path kernels are compiled once per
// mode, in parallel. RS_TU undefined: everything in one unit (tools/regs.sh, build_variant.sh);
// RS_TU = -1: the common unit (mode-independent kernels, the launchers that dispatch on the scene
// mode); RS_TU = k >= 0: scene mode k's launch_*_sm<k> instantiations only.
#if !defined(RS_TU)
#define RS_TU_COMMON 1
#define RS_TU_MODES 1
#elif RS_TU < 0
#define RS_TU_COMMON 1
#define RS_TU_MODES 0
#else
#define RS_TU_COMMON 0
#define RS_TU_MODES 1
#endif

// the streaming (material-sorted) wavefront's scene modes (rs_internal.h streaming_mode)
#define RS_SM_SORTED_DISPATCH(sm, ...)                                     \
    do {                                                                   \
        switch (sm) {                                                      \
        case kSmNest0: { constexpr int SMC = kSmNest0; __VA_ARGS__; break; }     \
        case kSmNest2: { constexpr int SMC = kSmNest2; __VA_ARGS__; break; }     \
        default: { constexpr int SMC = kSmSpheres; __VA_ARGS__; break; }         \
        }                                                                  \
    } while (0)

// instantiate a launch for the scene mode (rs_internal.h SceneMode) as the constant SMC
#define RS_SM_DISPATCH(sm, ...)                                            \
    do {                                                                   \
        switch (sm) {                                                      \
        case kSmSpheres: { constexpr int SMC = kSmSpheres; __VA_ARGS__; break; } \
        case kSmFlat: { constexpr int SMC = kSmFlat; __VA_ARGS__; break; }       \
        case kSmNest0: { constexpr int SMC = kSmNest0; __VA_ARGS__; break; }     \
        case kSmNest2: { constexpr int SMC = kSmNest2; __VA_ARGS__; break; }     \
        default: { constexpr int SMC = kSmGeneric; __VA_ARGS__; break; }         \
        }                                                                  \
    } while (0)

namespace rs {

// Loads through an explicit global (address space 1) pointer: the scene arrays are reached through
// the DScene in device memory, so the compiler cannot infer their address space and emits flat
// loads with 64-bit address arithmetic per load. With the kernel-uniform base in SGPRs and a 32-bit
// byte offset these become `global_load ... v_off, s[base]` (one VGPR of address per load).
typedef float f4v __attribute__((ext_vector_type(4)));
typedef int i4v __attribute__((ext_vector_type(4)));
typedef double d2v __attribute__((ext_vector_type(2)));
#define RS_GLOBAL __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ T gld(const void* base, uint32_t byte_off) {
    return *(const RS_GLOBAL T*)((const RS_GLOBAL char*)base + byte_off);
}
// Tree-node loads: global (gld), or with the scene's LDS image (LOBJ, lds_scene) plain loads through
// the image's pointers, which derive from the __shared__ array: the compiler emits ds_read for them.
template <bool LOBJ, class T>
__device__ __forceinline__ T nld(const void* base, uint32_t byte_off) {
    if constexpr (LOBJ) return *(const T*)((const char*)base + byte_off);
    else return gld<T>(base, byte_off);
}

// A sample's radiance in a rad buffer, item-major (3 doubles per item): a path that ends deep in the frame
// writes its radiance to a scattered item, and the three channels then share one line (channel-major
// buffers took three: bench frame 7.58 -> 7.43 ms, profiles/r5/ab). k_accumulate reads them pixel-major.
__device__ __forceinline__ void put_rad(double* __restrict__ rad, uint64_t item, double r, double g, double b) {
    rad[3 * item] = r; rad[3 * item + 1] = g; rad[3 * item + 2] = b;
}

#ifdef RS_TRAV_STATS  // dev builds only (tools/build_variant.sh -DRS_TRAV_STATS): traversal counters
// [cat][k], cat 0 camera rays / bounce-synchronous rays, 1 the carried front run (light-sample rays), 2 the rest;
// [cat][8 + b]: rays with 8b .. 8b+7 node steps (b < 16, last = more). One array per translation unit (each
// mode's kernels are their own code object): rs_debug_trav_stats_<unit> reads that unit's.
__device__ unsigned long long g_trav_stats[4][32];
#define RS_STAT(k, v) atomicAdd(&g_trav_stats[st_cat][k], (unsigned long long)(v))
__shared__ int s_st_nodes[256], s_st_leaves[256], s_st_witer[256];
#endif

// aabb.rs:20-38 with inv = 1/d[i] precomputed per ray (the reference recomputes the same value
// per node). Branch-free form: max/min over the three axes is equivalent to the early-exit loop
// because t_min only grows and t_max only shrinks. This exact f64 test is applied to every
// object's own bbox before the object is intersected.
__device__ __forceinline__ bool slab64(const double lo[3], const double hi[3], const V3& o, const V3& inv, double tmin,
                                       double tmax) {
    double t0x = (lo[0] - o.x) * inv.x, t1x = (hi[0] - o.x) * inv.x;
    double t0y = (lo[1] - o.y) * inv.y, t1y = (hi[1] - o.y) * inv.y;
    double t0z = (lo[2] - o.z) * inv.z, t1z = (hi[2] - o.z) * inv.z;
    if (inv.x < 0.0) { double t = t0x; t0x = t1x; t1x = t; }
    if (inv.y < 0.0) { double t = t0y; t0y = t1y; t1y = t; }
    if (inv.z < 0.0) { double t = t0z; t0z = t1z; t1z = t; }
    const double a = fmax(fmax(fmax(tmin, t0x), t0y), t0z);
    const double b = fmin(fmin(fmin(tmax, t1x), t1y), t1z);
    return !(b <= a);
}

// Conservative f32 slab test for inner nodes: never rejects a box the exact f64 test of any
// descendant leaf would accept. Boxes are rounded outward on the host. The ray origin is shifted
// per axis by d = |o|*2^-20 + tiny (an expanded box [lo-d, hi+d] in effect), which absorbs the f32
// rounding of o and of the precomputed products o'*inv (each <= |o| 2^-24); t at a plane is then one
// FMA, t = lo*inv - (o+d)*inv. The remaining roundings (inv, fma) are relative and covered by a
// 2^-18 slack on the interval. |inv| is clamped to 1e30 so no inf*0 / inf-inf appears.
struct RayF {
    float inv[3], opi[3], omi[3];   // inv, (o+d)*inv, (o-d)*inv
};
__device__ __forceinline__ float nextup_f(float f) {  // f finite, not the largest float
    if (f == 0.0f) return 0x1p-149f;
    const unsigned u = __float_as_uint(f);
    return __uint_as_float(f > 0.0f ? u + 1u : u - 1u);
}
__device__ __forceinline__ float round_up_f(double x) {
    const float f = (float)x;
    return ((double)f < x) ? nextup_f(f) : f;
}
__device__ __forceinline__ RayF make_rayf(const V3& o, const V3& inv) {
    RayF r;
    const double oo[3] = {o.x, o.y, o.z}, ii[3] = {inv.x, inv.y, inv.z};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float of = (float)oo[k];
        const float d = fabsf(of) * 0x1p-20f + 0x1p-100f;
        const float iv = fminf(fmaxf((float)ii[k], -1e30f), 1e30f);
        r.inv[k] = iv;
        r.opi[k] = (of + d) * iv;
        r.omi[k] = (of - d) * iv;
    }
    return r;
}
__device__ __forceinline__ bool slab32(const float lo[3], const float hi[3], const RayF& r, float tmin, float tmax,
                                       float& entry) {
    const float ax = fmaf(lo[0], r.inv[0], -r.opi[0]), bx = fmaf(hi[0], r.inv[0], -r.omi[0]);
    const float ay = fmaf(lo[1], r.inv[1], -r.opi[1]), by = fmaf(hi[1], r.inv[1], -r.omi[1]);
    const float az = fmaf(lo[2], r.inv[2], -r.opi[2]), bz = fmaf(hi[2], r.inv[2], -r.omi[2]);
    float a = fmaxf(fmaxf(fmaxf(tmin, fminf(ax, bx)), fminf(ay, by)), fminf(az, bz));
    float b = fminf(fminf(fminf(tmax, fmaxf(ax, bx)), fmaxf(ay, by)), fmaxf(az, bz));
    a = fmaf(-fabsf(a), 0x1p-18f, a);
    b = fmaf(fabsf(b), 0x1p-18f, b);
    entry = a;
    return a <= b;
}

// 4-wide nodes: the ray's direction signs pick, per axis, which of the node's lo / hi planes is
// the entry plane -- for inv >= 0 min(ax, bx) is ax (lo with o+d), else bx (hi with o-d), exactly
// (fma is monotone in each operand) -- so a child costs 6 FMAs and four min / max instead of the
// pairwise min / max of slab32. The plane arrays are fetched at per-ray byte offsets in DNode4.
struct RayF4 {
    float inv[3], nsub[3], fsub[3];   // entry / exit plane offsets ((o+d)*inv or (o-d)*inv)
    uint32_t noff[3];                 // byte offset of the entry-plane array (lo_* or hi_*)
};
__device__ __forceinline__ RayF4 make_rayf4(const RayF& r) {
    RayF4 q;
    constexpr uint32_t lo_off[3] = {0, 16, 32}, hi_off[3] = {48, 64, 80};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const bool pos = r.inv[k] >= 0.0f;
        q.inv[k] = r.inv[k];
        q.nsub[k] = pos ? r.opi[k] : r.omi[k];
        q.fsub[k] = pos ? r.omi[k] : r.opi[k];
        q.noff[k] = pos ? lo_off[k] : hi_off[k];
    }
    return q;
}
// the exit-plane array is the other one of the axis: lo_off ^ hi_off = 48, 80, 112
__device__ __forceinline__ uint32_t far_off(uint32_t noff, int k) { return noff ^ (k == 0 ? 48u : k == 1 ? 80u : 112u); }
__device__ __forceinline__ bool slab4(float nx, float ny, float nz, float fx, float fy, float fz, const RayF4& r,
                                      float tmin, float tmax, float& entry) {
    const float ax = fmaf(nx, r.inv[0], -r.nsub[0]), bx = fmaf(fx, r.inv[0], -r.fsub[0]);
    const float ay = fmaf(ny, r.inv[1], -r.nsub[1]), by = fmaf(fy, r.inv[1], -r.fsub[1]);
    const float az = fmaf(nz, r.inv[2], -r.nsub[2]), bz = fmaf(fz, r.inv[2], -r.fsub[2]);
    float a = fmaxf(fmaxf(fmaxf(tmin, ax), ay), az);
    float b = fminf(fminf(fminf(tmax, bx), by), bz);
    a = fmaf(-fabsf(a), 0x1p-18f, a);
    b = fmaf(fabsf(b), 0x1p-18f, b);
    entry = a;
    return a <= b;
}
// One 4-wide node's planes for the ray: per axis the entry (N*) and exit (F*) plane of the four child
// boxes, fetched at the per-ray byte offsets of the ray's direction signs, and the child codes. (A 64-byte
// node with half-float planes, rounded outward, the whole node in four loads and the arrays selected and
// widened in registers, measured 3 % slower on the bench frame and equal on the C5 mesh: round 4.)
template <bool LOBJ = false>
__device__ __forceinline__ void load_node4(const DScene& S, const RayF4& rq, int node, f4v& NX, f4v& FX, f4v& NY, f4v& FY,
                                           f4v& NZ, f4v& FZ, i4v& NC) {
    const uint32_t nb = (uint32_t)node * (uint32_t)sizeof(DNode4);  // < 4 GiB of nodes (host-checked)
    NX = nld<LOBJ, f4v>(S.nodes4, nb + rq.noff[0]); FX = nld<LOBJ, f4v>(S.nodes4, nb + far_off(rq.noff[0], 0));
    NY = nld<LOBJ, f4v>(S.nodes4, nb + rq.noff[1]); FY = nld<LOBJ, f4v>(S.nodes4, nb + far_off(rq.noff[1], 1));
    NZ = nld<LOBJ, f4v>(S.nodes4, nb + rq.noff[2]); FZ = nld<LOBJ, f4v>(S.nodes4, nb + far_off(rq.noff[2], 2));
    NC = nld<LOBJ, i4v>(S.nodes4, nb + 96u);
}

// Test one leaf object with the range [tmin, best); on acceptance best := its t1 (the
// reference's right subtree is searched with `start..left.t1`, bvh.rs:179-188, i.e. the last
// accepted hit sets the range end, which is the minimum except for Difference's back-face hits).
// Sphere leaf during traversal: same arithmetic as sphere_t (sphere.rs:83-109) with the per-ray
// a = |d|^2 hoisted and center_at skipped for static spheres (c + 0*t == c bit for bit).
__device__ __forceinline__ bool sphere_t_trav(const DSphere& s, const Ray& r, double a, double tmin, double tmax,
                                              double& t, bool moving = true) {
    V3 cc = ld3(s.c);
    if (moving && (s.v[0] != 0.0 || s.v[1] != 0.0 || s.v[2] != 0.0)) cc = cc + ld3(s.v) * r.time;
    const V3 l = r.o - cc;
    const double half_b = dot(r.d, l);
    const double c = len2(l) - s.r2;
    const double delta = half_b * half_b - a * c;
    if (delta < 0.0) return false;
    const double sq = sqrt(delta);
    const double t1 = (-half_b - sq) / a;
    if (in_range(t1, tmin, tmax)) { t = t1; return true; }
    const double t2 = (-half_b + sq) / a;
    if (in_range(t2, tmin, tmax)) { t = t2; return true; }
    return false;
}

// Per-ray constants of the leaf tests, computed once per traversal: inv = 1 / d (the value
// AABB::hit computes per node, aabb.rs:24) and a = |d|^2 (Sphere::hit's `a`, sphere.rs:88).
struct RayC {
    V3 inv;
    double a;
};
__device__ __forceinline__ RayC ray_consts(const Ray& r) {
    RayC c;
    c.inv = v3(1.0 / r.d.x, 1.0 / r.d.y, 1.0 / r.d.z);
    c.a = len2(r.d);
    return c;
}
// The same constants computed where this is called: the direction goes through an empty asm first, so
// the compiler cannot merge two branches' copies and hoist the three f64 divisions above the branch
// (the flat leaf test needs them only for an accepted triangle; hoisted, they ran before every leaf's loads)
__device__ __forceinline__ RayC ray_consts_here(const Ray& r) {
    V3 d = r.d;
    asm volatile("" : "+v"(d.x), "+v"(d.y), "+v"(d.z));
    RayC c;
    c.inv = v3(1.0 / d.x, 1.0 / d.y, 1.0 / d.z);
    c.a = len2(d);
    return c;
}

// A sphere record through global loads; the speed only in scenes with moving spheres
// (DScene::moving: static spheres skip c + v*t, which is c bit for bit for v = 0)
__device__ __forceinline__ DSphere ld_sphere(const DScene& S, const DSphere* arr, int i) {
    const uint32_t o = (uint32_t)i * (uint32_t)sizeof(DSphere);
    const d2v a = gld<d2v>(arr, o), b = gld<d2v>(arr, o + 16);
    DSphere s;
    s.c[0] = a.x; s.c[1] = a.y; s.c[2] = b.x; s.r = b.y;
    s.r2 = gld<double>(arr, o + 32);
    if (S.moving) {
        s.v[0] = gld<double>(arr, o + 40);
        const d2v c = gld<d2v>(arr, o + 48);
        s.v[1] = c.x; s.v[2] = c.y;
    } else {
        s.v[0] = s.v[1] = s.v[2] = 0.0;
    }
    return s;
}

// A static sphere from its 32-byte record: r2 = r * r is radius_squared's own f64 product (sphere.rs:40)
__device__ __forceinline__ DSphere ld_sphere_s(const DSphereS* arr, int i) {
    const uint32_t o = (uint32_t)i * (uint32_t)sizeof(DSphereS);
    const d2v a = gld<d2v>(arr, o), b = gld<d2v>(arr, o + 16);
    DSphere s;
    s.c[0] = a.x; s.c[1] = a.y; s.c[2] = b.x; s.r = b.y;
    s.r2 = s.r * s.r;
    s.v[0] = s.v[1] = s.v[2] = 0.0;
    return s;
}

// A leaf-ordered triangle record (80 B) through five 16-byte global loads
__device__ __forceinline__ LTri ld_ltri(const LTri* arr, int i) {
    const uint32_t o = (uint32_t)i * (uint32_t)sizeof(LTri);
    const d2v a = gld<d2v>(arr, o), b = gld<d2v>(arr, o + 16), c = gld<d2v>(arr, o + 32), d = gld<d2v>(arr, o + 48),
              f = gld<d2v>(arr, o + 64);
    // all five in registers here: the callers branch on `kind` (the last 16 B) first, and the compiler
    // would otherwise sink the other four loads into the triangle branch -- a second dependent L2 round
    // trip per leaf test
    asm volatile("" ::"v"(a), "v"(b), "v"(c), "v"(d), "v"(f));
    LTri T;
    T.p0[0] = a.x; T.p0[1] = a.y; T.p0[2] = b.x; T.a = b.y; T.b = c.x; T.c = c.y; T.d = d.x; T.e = d.y; T.f = f.x;
    T.kind = f.y;
    return T;
}

// Sphere leaf (leaf entry e): discriminant first, then the exact own box for spheres that hit.
__device__ __forceinline__ void test_sphere_leaf(const DScene& S, const DSphere& sp, int e, const Ray& r, const RayC& rc,
                                                 double tmin, double& best, double& bend, int& bp) {
    double t;
#ifdef RS_LEAF_TWICE  // dev bound (tools/build_variant.sh): the quadratic done twice, the copy's inputs opaque
    {
        DSphere s2 = sp;
        asm volatile("" : "+v"(s2.c[0]), "+v"(s2.c[1]), "+v"(s2.c[2]), "+v"(s2.r2));
        double t2;
        const bool h2 = sphere_t_trav(s2, r, rc.a, tmin, best, t2, S.moving != 0);
        asm volatile("" ::"v"(t2), "v"((int)h2));
    }
#endif
    if (!sphere_t_trav(sp, r, rc.a, tmin, best, t, S.moving != 0)) return;
    double lo[3], hi[3];
    if (!S.moving || (sp.v[0] == 0.0 && sp.v[1] == 0.0 && sp.v[2] == 0.0)) {  // host: c -/+ r (sphere.rs:117-124)
        lo[0] = sp.c[0] - sp.r; lo[1] = sp.c[1] - sp.r; lo[2] = sp.c[2] - sp.r;
        hi[0] = sp.c[0] + sp.r; hi[1] = sp.c[1] + sp.r; hi[2] = sp.c[2] + sp.r;
    } else {
        const DBox64& B = S.pbox[S.lprim ? S.lprim[e] : e];
        lo[0] = B.lo[0]; lo[1] = B.lo[1]; lo[2] = B.lo[2]; hi[0] = B.hi[0]; hi[1] = B.hi[1]; hi[2] = B.hi[2];
    }
    if (!slab64(lo, hi, r.o, rc.inv, tmin, best)) return;
    bend = best; best = t; bp = e;
}

// Nested-object entry points: Obj<L> instantiated only as deep as the scene mode needs.
template <int SM>
__device__ __forceinline__ bool obj_hit(const DScene& S, int p, const Ray& r, double tmin, double tmax, Hit& h) {
    return Obj<nest_of(SM), rich_of(SM)>::hit(S, p, r, tmin, tmax, h);
}
template <int SM>
__device__ __forceinline__ bool obj_hit_t(const DScene& S, int p, const Ray& r, double tmin, double tmax, HitT& h) {
    return Obj<nest_of(SM), rich_of(SM)>::hit_t(S, p, r, tmin, tmax, h);
}
template <int SM>
__device__ __forceinline__ V3 obj_random(const DScene& S, int p, V3 origin, Rng& rng) {
    return Obj<nest_of(SM), rich_of(SM)>::random(S, p, origin, rng);
}

// Object hit for flat scenes (spheres, rects, triangles; no nesting): Obj<L>::hit's leaf cases only.
// uv: compute the record's (u, v) (the winner's record when the scene reads them; never in traversal)
__device__ __forceinline__ bool flat_hit(const DScene& S, const DPrim& P, const Ray& r, double tmin, double tmax, Hit& h,
                                         int uv = 0) {
    if (P.kind == PK_TRIANGLE) return tri_hit(S.tris[P.idx], P.mat, r, tmin, tmax, h);
    if (P.kind == PK_RECT) {
        const DRect& R = S.rects[P.idx];
        return rect_hit_raw(R.ax0, R.ax1, R.ax2, R.k, R.a0, R.a1, R.b0, R.b1, P.mat, r, tmin, tmax, h, uv);
    }
    return sphere_hit(S.spheres[P.idx], P.mat, r, tmin, tmax, h, uv);
}

// Leaf entry e: its object is accepted iff its exact own bbox passes (aabb.rs:20-38, BVH leaf box)
// AND it hits within [tmin, best). Both are pure, so the cheap test runs first: for spheres the
// discriminant, for triangles the barycentric test, and the exact box only for those that hit.
// On acceptance bp := e (traverse maps the winning entry to its prim handle at the end).
template <int SM, bool LOBJ = false>
__device__ __forceinline__ void test_leaf(const DScene& S, int e, const Ray& r, const RayC& rc, double tmin, double& best,
                                          double& bend, int& bp) {
    if (SM == kSmSpheres) {  // prim-indexed sphere copy: no DPrim hop (e is the prim in this mode)
        test_sphere_leaf(S, S.moving ? ld_sphere(S, S.lsph, e) : ld_sphere_s(S.lsphs, e), e, r, rc, tmin, best, bend, bp);
        return;
    }
    if (SM == kSmFlat) {  // leaf-ordered triangle copy; its `kind` field says whether entry e is one
        const LTri T = ld_ltri(S.ltri, e);
        if (T.kind == (double)PK_TRIANGLE) {
            double t;
            if (!tri_t(T, r, tmin, best, t)) return;
            // the ray constants are recomputed here (accepted triangles only) instead of being kept
            // live through the traversal: flat-scene extend runs at 5 waves on a 96-VGPR budget
            const RayC lc = ray_consts_here(r);
            const DBox64& B = S.pbox[S.lprim[e]];
            if (!slab64(B.lo, B.hi, r.o, lc.inv, tmin, best)) return;
            bend = best; best = t; bp = e;
            return;
        }
        const int p = S.lprim[e];
        const DPrim P = S.prims[p];
        const RayC lc = ray_consts_here(r);
        if (P.kind == PK_SPHERE) {
            test_sphere_leaf(S, S.spheres[P.idx], e, r, lc, tmin, best, bend, bp);
        } else {
            const DBox64& B = S.pbox[p];
            if (!slab64(B.lo, B.hi, r.o, lc.inv, tmin, best)) return;
            Hit tmp;
            if (flat_hit(S, P, r, tmin, best, tmp)) { bend = best; best = tmp.t1; bp = e; }
        }
        return;
    }
    const int p = S.lprim ? S.lprim[e] : e;  // nest / generic scenes' leaves name prims directly
    const DPrim P = S.prims[p];
    if (P.kind == PK_SPHERE) {
        test_sphere_leaf(S, S.spheres[P.idx], e, r, rc, tmin, best, bend, bp);
    } else {
        const DBox64& B = S.pbox[p];
        if (!slab64(B.lo, B.hi, r.o, rc.inv, tmin, best)) return;
        HitT tmp;  // t1 decides; the winner's record is built once, after the traversal (finish_hit)
        if (obj_hit_t<SM>(S, p, r, tmin, best, tmp)) { bend = best; best = tmp.t1; bp = e; }
    }
}

// World::hit (world.rs:63-65) -> BVH::hit (bvh.rs:173-192). Every object sits in its own leaf
// whose box is the object's own bbox. Two visiting orders:
//  * near-first (ref_order = 0): for scenes whose objects all return the closest root in range
//    (spheres, rects, triangles and transforms of them) the result is order independent;
//  * reference order (ref_order = 1): left subtree completely, then the right one with the
//    updated range -- needed for Box / Quadric / CSG, whose records depend on the range end.
//    Each child box is tested when the recursion would visit it (the deferred right child is
//    re-read from its parent when popped), so the tests see the same range as BVH::hit.
// Traversal stack of one thread: entries [0, kStackMax) in its column of the block's LDS stack
// (stride kBlock), deeper ones in its column of the HBM overflow array (stride = grid threads).
// The host sizes the overflow from the tree's exact worst-case depth, so any tree depth works;
// scenes whose trees fit the LDS part never touch HBM (the bound test is one compare per push/pop).
// The overflow address is formed only on the (rare) deep path, from the kernel-uniform base and the
// thread's grid index, so the common path keeps no extra registers live.
// OVF = false: the host guarantees stack_need + 3 <= kStackMax (no HBM part; the bvh4 push's three
// unconditional writes stay inside the LDS column), so push / pop are plain LDS accesses.
// N: the entries of the LDS part (stack_lds); the overflow rows start at entry N (the host sizes
// them for the smallest N, kStackMin)
template <bool OVF, int N = kStackMax>
struct StkT {
    static constexpr bool kOvf = OVF;
    static constexpr int kN = N;
    int* lds;          // this thread's column of the block's LDS stack
    int* ovf_base;     // DScene::stk_ovf (uniform)
    __device__ __forceinline__ int* ovf(int i) const {
        return ovf_base + ((size_t)(i - N) * gridDim.x * kBlock + (size_t)blockIdx.x * kBlock + threadIdx.x);
    }
    __device__ __forceinline__ void put(int i, int v) const {
        if (!OVF || i < N) lds[i * kBlock] = v;
        else *ovf(i) = v;
    }
    __device__ __forceinline__ int get(int i) const { return (!OVF || i < N) ? lds[i * kBlock] : *ovf(i); }
};
using Stk = StkT<true>;
// this thread's stack (stk_all = the block's LDS array of N x kBlock entries)
template <bool OVF = true, int N = kStackMax>
__device__ __forceinline__ StkT<OVF, N> make_stk(const DScene& S, int* stk_all) {
    StkT<OVF, N> s;
    s.lds = stk_all + threadIdx.x;
    s.ovf_base = S.stk_ovf;
    return s;
}
#ifdef RS_TRAV_STATS
// all 64 lanes converged: per ray sums, per wave the max node count (the wave runs the union of its
// lanes' loops) and the wave's live lanes
__device__ __forceinline__ void trav_stats_flush(bool live, int st_cat = 0) {
    int n = live ? s_st_nodes[threadIdx.x] : 0, l = live ? s_st_leaves[threadIdx.x] : 0, mx = n, cnt = live ? 1 : 0;
    for (int off = 32; off > 0; off >>= 1) {
        n += __shfl_xor(n, off, 64); l += __shfl_xor(l, off, 64); cnt += __shfl_xor(cnt, off, 64);
        mx = max(mx, __shfl_xor(mx, off, 64));
    }
    int wi = live ? s_st_witer[threadIdx.x] : 0;  // the wave's leaf-loop passes: the max over its lanes
    for (int off = 32; off > 0; off >>= 1) wi = max(wi, __shfl_xor(wi, off, 64));
    if ((threadIdx.x & 63) == 0 && cnt) { RS_STAT(0, n); RS_STAT(1, l); RS_STAT(2, cnt); RS_STAT(3, mx); RS_STAT(4, cnt); RS_STAT(5, 1); RS_STAT(6, wi); }
    if (live) RS_STAT(8 + min(15, max(0, s_st_nodes[threadIdx.x]) / 8), 1);
}
#endif
// One node of the 4-wide near-first traversal: test the four child boxes of one 128-byte node,
// push the farther inner children, test the node's leaves; returns the next node (-1: done).
// Shared by traverse() and the persistent-lane flat-scene extend (k_wf_extend_pl).
#ifdef RS_TRAV_STATS
#define RS_ST_PARAMS , int& st_leaves, int& st_witer
#define RS_ST_PASS , st_leaves, st_witer
#else
#define RS_ST_PARAMS
#define RS_ST_PASS
#endif
// The spheres mode's tree top in LDS (TOP): the extend's blocks copy nodes 0 .. S.ltop - 1 of the breadth-first
// tree here; a node step whose wave is entirely inside the top reads its node with ds_read (a wave-uniform choice,
// so no lane waits on both paths), the others from the global copy.
__shared__ DNode4 s_top4[kLTop > 0 ? kLTop : 1];
template <int SM, class STK, bool LOBJ = false, bool TOP = false>
__device__ __forceinline__ int bvh4_step(const DScene& S, const Ray& r, const RayC& rc, const RayF4& rq, double tmin,
                                 float tmin32, int node, int& sp, const STK& stk, double& best, double& bend,
                                 int& bp, float& best32 RS_ST_PARAMS) {
#ifdef RS_TRAV_STATS
#define RS_ST_LEAF4() ++st_leaves
#else
#define RS_ST_LEAF4()
#endif
#define RS_LEAF4(code)                                                         \
    do {                                                                       \
        RS_ST_LEAF4();                                                         \
        const int bp_prev = bp;                                                \
        test_leaf<SM, LOBJ>(S, ~(code), r, rc, tmin, best, bend, bp);          \
        if (bp != bp_prev || bp >= 0) best32 = round_up_f(best);               \
    } while (0)
    f4v NX, FX, NY, FY, NZ, FZ;
    i4v NC;
    if (TOP && __ballot(node >= S.ltop) == 0ull) {
        DScene T = S;
        T.nodes4 = s_top4;
        load_node4<true>(T, rq, node, NX, FX, NY, FY, NZ, FZ, NC);
    } else {
        load_node4<LOBJ>(S, rq, node, NX, FX, NY, FY, NZ, FZ, NC);
    }
    // per slot: inner-child code and entry (or -inf = not to visit); leaf codes are collected
    // and tested after the four box tests, when the node's registers are dead. Branch-free:
    // all four boxes are tested (the node's loads issue together) and the slot results are
    // selects; an empty slot (INT32_MIN) is neither a leaf nor an inner child.
    int n0, n1, n2, n3, l0, l1, l2, l3;
    float e0, e1, e2, e3;
#define RS_SLOT(K, NK, EK, LK)                                                                \
    {                                                                                 \
        float e;                                                                      \
        const int c = NC.K;                                                           \
        const bool hk = slab4(NX.K, NY.K, NZ.K, FX.K, FY.K, FZ.K, rq, tmin32, best32, e) & (c != INT32_MIN); \
        LK = (hk & (c < 0)) ? c : INT32_MIN;                                          \
        NK = c;                                                                       \
        EK = (hk & (c >= 0)) ? e : -__builtin_huge_valf();                            \
    }
    RS_SLOT(x, n0, e0, l0) RS_SLOT(y, n1, e1, l1) RS_SLOT(z, n2, e2, l2) RS_SLOT(w, n3, e3, l3)
#undef RS_SLOT
#ifdef RS_TRAV_STATS
    {   // leaf-loop passes of the wave at this node (the active lanes' maximum leaf count)
        const int nl = (l0 != INT32_MIN) + (l1 != INT32_MIN) + (l2 != INT32_MIN) + (l3 != INT32_MIN);
        for (int q = 1; q <= 4; ++q) st_witer += __ballot(nl >= q) != 0ull;
    }
#endif
    const int cnt = (e0 > -__builtin_huge_valf()) + (e1 > -__builtin_huge_valf()) +
                    (e2 > -__builtin_huge_valf()) + (e3 > -__builtin_huge_valf());
    int next = -1;
    if (cnt > 0) {
        // sort descending by entry (farthest first, not-visited last): 5 compare-swaps
#define RS_CS(EA, NA, EB, NB) if (EB > EA) { const float te = EA; EA = EB; EB = te; const int tn = NA; NA = NB; NB = tn; }
        RS_CS(e0, n0, e1, n1) RS_CS(e2, n2, e3, n3) RS_CS(e0, n0, e2, n2) RS_CS(e1, n1, e3, n3) RS_CS(e1, n1, e2, n2)
#undef RS_CS
        // the cnt - 1 farther children are pushed; inside the LDS part all three writes are
        // issued (the ones above sp + cnt - 1 are dead), near its end only the live ones
        if (!STK::kOvf || sp + 3 <= STK::kN) {
            stk.lds[sp * kBlock] = n0;
            stk.lds[(sp + 1) * kBlock] = n1;
            stk.lds[(sp + 2) * kBlock] = n2;
        } else {
            if (cnt > 1) stk.put(sp, n0);
            if (cnt > 2) stk.put(sp + 1, n1);
            if (cnt > 3) stk.put(sp + 2, n2);
        }
        sp += cnt - 1;
        next = cnt == 1 ? n0 : cnt == 2 ? n1 : cnt == 3 ? n2 : n3;
    }
    // leaves of this node (their hits only shrink the range the next node is tested with),
    // in slot order through ONE copy of the leaf test: every lane tests its k-th leaf in
    // the same pass, so a wave runs max-over-lanes leaf tests per node, not one pass per
    // slot that any lane uses (one `if` per slot measured 2 % slower)
    while (true) {
        int code;
        if (l0 != INT32_MIN) { code = l0; l0 = INT32_MIN; }
        else if (l1 != INT32_MIN) { code = l1; l1 = INT32_MIN; }
        else if (l2 != INT32_MIN) { code = l2; l2 = INT32_MIN; }
        else if (l3 != INT32_MIN) { code = l3; l3 = INT32_MIN; }
        else break;
        RS_LEAF4(code);
    }
    if (cnt == 0 && sp > 0) {
        --sp;
        next = stk.get(sp);
    }
    return next;
#undef RS_LEAF4
#undef RS_ST_LEAF4
}


// ---- flat scenes (meshes): node steps and leaf tests in separate wave passes ----
// In bvh4_step a wave runs each node's leaf loop as long as the lane with the most leaves there, and
// its other lanes idle through the f64 triangle tests (the lanes' divergence sits inside the node
// steps). Here a lane's leaf entries go to a FIFO of RS_LEAFQ entries in LDS instead, and the wave
// chooses, pass by pass: a leaf pass (every lane with a queued entry tests its oldest one) when at
// least RS_LEAFQ_THR/64 of its working lanes have one queued or no lane can take a node step;
// otherwise a node step for the lanes with room for four more entries. The choice is wave-uniform
// (ballots), so neither pass diverges on it.
// Same hit as traverse(): a lane tests its entries in the order it met them, only later (a node step
// culls with the range the tests so far left, a superset of the nodes bvh4_step visits), and flat
// scenes' objects are monotone -- a later test sees a range at least as large, the closest entry wins
// whatever the order (equal t: the first met, as before), and the winner's record needs only a range
// end above its own t.
#define RS_LEAFQ 8      // entries per lane (power of two, >= 8)
#ifndef RS_LEAFQ_THR
#define RS_LEAFQ_THR 48  // leaf pass at >= 48/64 of the working lanes with an entry queued (with the lane refill:
                         // 32 / 40 / 56 -> +0.8 / -0.1 / +1.9 % of the mesh extend, profiles/r5/ab/c5_leafq_thr_r6h.jsonl)
#endif
template <int SM, class STK>
__device__ __forceinline__ int bvh4_node_q(const DScene& S, const RayF4& rq, float tmin32, float best32, int node, int& sp,
                                           const STK& stk, int* q, int& qt) {
    f4v NX, FX, NY, FY, NZ, FZ;
    i4v NC;
    load_node4(S, rq, node, NX, FX, NY, FY, NZ, FZ, NC);
    int n0, n1, n2, n3, l0, l1, l2, l3;
    float e0, e1, e2, e3;
#define RS_SLOT(K, NK, EK, LK)                                                                \
    {                                                                                 \
        float e;                                                                      \
        const int c = NC.K;                                                           \
        const bool hk = slab4(NX.K, NY.K, NZ.K, FX.K, FY.K, FZ.K, rq, tmin32, best32, e) & (c != INT32_MIN); \
        LK = (hk & (c < 0)) ? c : INT32_MIN;                                          \
        NK = c;                                                                       \
        EK = (hk & (c >= 0)) ? e : -__builtin_huge_valf();                            \
    }
    RS_SLOT(x, n0, e0, l0) RS_SLOT(y, n1, e1, l1) RS_SLOT(z, n2, e2, l2) RS_SLOT(w, n3, e3, l3)
#undef RS_SLOT
    // the leaf entries, in slot order, to the lane's FIFO: four unconditional writes at the tail (the
    // caller guarantees four free entries), the tail advanced past the real ones
    {
        constexpr int M = RS_LEAFQ - 1;
        int k = qt;
        q[(k & M) * kBlock] = l0; k += l0 != INT32_MIN;
        q[(k & M) * kBlock] = l1; k += l1 != INT32_MIN;
        q[(k & M) * kBlock] = l2; k += l2 != INT32_MIN;
        q[(k & M) * kBlock] = l3; k += l3 != INT32_MIN;
        qt = k;
    }
    const int cnt = (e0 > -__builtin_huge_valf()) + (e1 > -__builtin_huge_valf()) +
                    (e2 > -__builtin_huge_valf()) + (e3 > -__builtin_huge_valf());
    int next;
    if (cnt == 0) {
        next = -1;
        if (sp > 0) { --sp; next = stk.get(sp); }
    } else {
#define RS_CS(EA, NA, EB, NB) if (EB > EA) { const float te = EA; EA = EB; EB = te; const int tn = NA; NA = NB; NB = tn; }
        RS_CS(e0, n0, e1, n1) RS_CS(e2, n2, e3, n3) RS_CS(e0, n0, e2, n2) RS_CS(e1, n1, e3, n3) RS_CS(e1, n1, e2, n2)
#undef RS_CS
        if (!STK::kOvf || sp + 3 <= STK::kN) {
            stk.lds[sp * kBlock] = n0;
            stk.lds[(sp + 1) * kBlock] = n1;
            stk.lds[(sp + 2) * kBlock] = n2;
        } else {
            if (cnt > 1) stk.put(sp, n0);
            if (cnt > 2) stk.put(sp + 1, n1);
            if (cnt > 3) stk.put(sp + 2, n2);
        }
        sp += cnt - 1;
        next = cnt == 1 ? n0 : cnt == 2 ? n1 : cnt == 3 ? n2 : n3;
    }
    return next;
}

// World::hit of a flat scene with a 4-wide tree through queued leaf passes (above). q: this lane's
// column of the block's FIFO array (RS_LEAFQ x kBlock ints). Every lane of the wave that calls it
// must call it (the pass choice is a ballot over the calling lanes).
template <int SM, class STK>
__device__ __forceinline__ int traverse_flat_q(const DScene& S, const Ray& r, double tmin, double& bend_out, const STK& stk,
                                               int* q) {
    const RayC rc = ray_consts(r);
    const RayF4 rq = make_rayf4(make_rayf(r.o, rc.inv));
    const float tmin32 = -round_up_f(-tmin);
    double best = RS_INF, bend = RS_INF;
    float best32 = __builtin_huge_valf();
    int bp = -1, node = S.root4, sp = 0, qh = 0, qt = 0;
#ifdef RS_TRAV_STATS
    int st_nodes = 0, st_leaves = 0, st_witer = 0;
#endif
    while (true) {
        const bool has_leaf = qt != qh;
        const bool can_node = node >= 0 && qt - qh <= RS_LEAFQ - 4;
        const uint64_t work = __ballot(node >= 0 || has_leaf);
        if (work == 0ull) break;
        const uint64_t lm = __ballot(has_leaf);
        if (__popcll(lm) * 64 >= RS_LEAFQ_THR * __popcll(work) || __ballot(can_node) == 0ull) {
#ifdef RS_TRAV_STATS
            ++st_witer;
#endif
            if (has_leaf) {
                const int code = q[(qh & (RS_LEAFQ - 1)) * kBlock];
                ++qh;
#ifdef RS_TRAV_STATS
                ++st_leaves;
#endif
                const int bp_prev = bp;
                test_leaf<SM>(S, ~code, r, rc, tmin, best, bend, bp);
                if (bp != bp_prev || bp >= 0) best32 = round_up_f(best);
            }
        } else if (can_node) {
#ifdef RS_TRAV_STATS
            ++st_nodes;
#endif
            node = bvh4_node_q<SM>(S, rq, tmin32, best32, node, sp, stk, q, qt);
        }
    }
#ifdef RS_TRAV_STATS
    s_st_nodes[threadIdx.x] = st_nodes;
    s_st_leaves[threadIdx.x] = st_leaves;
    s_st_witer[threadIdx.x] = st_witer;
#endif
    bend_out = bend;
    return (bp >= 0 && S.lprim) ? S.lprim[bp] : bp;
}

// World::hit in BVH::hit's recursion order (bvh.rs:173-192) on the in-order 4-wide tree with the leaf
// tests taken out of the walk: the walk lists the leaves whose boxes the ray reaches in [tmin, inf), in
// the recursion's order, kLeafBatch at a time into the top of the thread's LDS stack column, and the
// listed leaves are then tested in that order with the range so far. Same hits as the interleaved walk:
// the range only culls (a leaf is accepted iff its own exact box passes with the range of its turn and
// it hits, and the walk's order does not depend on the range), and the list holds every leaf the
// interleaved walk would test, in order. The walk's and the tests' registers are never live together.
// A ray with more leaves walks again
// for the next kLeafBatch (the LDS-image scenes' trees are a few nodes). The host gives a scene its LDS
// image only when stack_need + kLeafBatch <= stack_lds(mode) and the tree is the in-order 4-wide one.
template <int SM, class STK>
__device__ __forceinline__ int traverse_deferred(const DScene& S, const Ray& r, double tmin, double& bend_out, const STK& stk) {
    constexpr uint32_t K = kLeafBatch;
    int* const q = stk.lds + (STK::kN - (int)K) * kBlock;  // this thread's list slots
    const RayC rc = ray_consts(r);
    const float tmin32 = -round_up_f(-tmin);
    double best = RS_INF, bend = RS_INF;
    int bp = -1;
    uint32_t skip = 0;
#ifdef RS_TRAV_STATS
    int st_nodes = 0, st_leaves = 0;
#endif
    while (true) {
        uint32_t found = 0;  // leaves met by this walk; slots skip .. skip + K - 1 are listed
        {
            const RayF rf = make_rayf(r.o, rc.inv);
            int k = 0, node = S.root4, sp = 0;
            while (true) {
                const uint32_t nb = (uint32_t)node * (uint32_t)sizeof(DNode4) + 4u * (uint32_t)k;
                const int c = nld<true, int>(S.nodes4, nb + 96u);
                if (c == INT32_MIN) {  // slots are filled from the left: the node is done
                    if (sp == 0) break;
                    --sp;
                    const int v = stk.get(sp);
                    node = v >> 2; k = v & 3;
                    continue;
                }
                const float lo[3] = {nld<true, float>(S.nodes4, nb), nld<true, float>(S.nodes4, nb + 16u),
                                     nld<true, float>(S.nodes4, nb + 32u)};
                const float hi[3] = {nld<true, float>(S.nodes4, nb + 48u), nld<true, float>(S.nodes4, nb + 64u),
                                     nld<true, float>(S.nodes4, nb + 80u)};
                float e;
#ifdef RS_TRAV_STATS
                ++st_nodes;  // (deferred walk: box tests)
#endif
                if (slab32(lo, hi, rf, tmin32, __builtin_huge_valf(), e)) {
                    if (c < 0) {
                        if (found >= skip && found - skip < K) q[(found - skip) * kBlock] = c;
                        ++found;
                    } else {
                        if (k < 3) { stk.put(sp, node * 4 + k + 1); ++sp; }  // come back for the next slot
                        node = c;
                        k = 0;
                        continue;
                    }
                }
                if (k < 3) { ++k; continue; }
                if (sp == 0) break;
                --sp;
                const int v = stk.get(sp);
                node = v >> 2; k = v & 3;
            }
        }
        const uint32_t m = found > skip ? min(found - skip, K) : 0u;
#ifndef RS_NO_KIND_MAJOR
        // Kind-major leaf tests (nest-2): a wave's lanes list leaves of different kinds (sphere, box, a TfFacade
        // over a CSG, ...), and testing every lane's i-th leaf together runs the object code of every kind present
        // at position i. Here each step takes one kind -- the current leaf kind of the wave's first unfinished
        // lane -- and every lane whose current leaf has that kind tests it and the leaves after it while they
        // have the same kind. A lane still tests its own leaves in its listed order with the range the ones
        // before left (the same hits); a step never runs two kinds' code. C4-shaped frame: extend 71.3 -> 69.2
        // ms; nest-0 (example.sdl, cheap leaves) 7.37 -> 7.78 ms, so nest-0 keeps the position-major loop
        // (profiles/r5/ab/kind_major_r6a.jsonl).
        if constexpr (SM == kSmNest2) {
            uint32_t i = 0;
            int kd = m > 0 ? (int)S.prims[~q[0]].kind : -1;
            while (true) {
                const uint64_t act = __ballot(i < m);
                if (act == 0ull) break;
                const int kw = __shfl(kd, __ffsll((long long)act) - 1, 64);
                while (i < m && kd == kw) {
                    test_leaf<SM, true>(S, ~q[i * kBlock], r, rc, tmin, best, bend, bp);
                    ++i;
                    kd = i < m ? (int)S.prims[~q[i * kBlock]].kind : -1;
                }
            }
        } else
#endif
        for (uint32_t i = 0; i < m; ++i) test_leaf<SM, true>(S, ~q[i * kBlock], r, rc, tmin, best, bend, bp);
#ifdef RS_TRAV_STATS
        st_leaves += (int)m;
#endif
        if (found <= skip + K) break;
        skip += K;
    }
#ifdef RS_TRAV_STATS
    s_st_nodes[threadIdx.x] = st_nodes;
    s_st_leaves[threadIdx.x] = st_leaves;
    s_st_witer[threadIdx.x] = 0;
#endif
    bend_out = bend;
    return bp;  // nest modes' leaf codes name prims (no lprim)
}

// World::hit, inlined into the kernels of every scene mode (a real call makes the kernel keep its live
// registers in scratch across it: the nest-2 extend spilled 1.2 KB per lane; the generic mode as a
// call measured slower in round 3, profiles/r3/ab/generic_inline_*.txt)
// TOUT: bend_out receives the winner's own t (best) instead of the range end it was accepted under (the spheres
// mode's shading rebuilds the record from t: sphere_rec_at)
template <int SM, class STK, bool LOBJ = false, bool TOUT = false, bool TOP = false>
__device__ __forceinline__ int traverse(const DScene& S, const Ray& r, double tmin, double& bend_out, const STK& stk) {
    if (S.root < 0) return -1;
    // the nest modes with an LDS image: example.sdl 2.5 % faster (profiles/r4/ab/deferred_leaves); C4's scene
    // 2 % slower in round 4, 14 % faster since the nested-object registers were cut (the walk's and the tests'
    // registers are never live together: scratch 184 -> 144 B at 3 waves; profiles/r5/ab/c4_variants_r5c.jsonl)
    if constexpr (LOBJ && (SM == kSmNest0 || SM == kSmNest2)) return traverse_deferred<SM>(S, r, tmin, bend_out, stk);
    const RayC rc = ray_consts(r);
    const RayF rf = make_rayf(r.o, rc.inv);
    const float tmin32 = -round_up_f(-tmin);
    double best = RS_INF, bend = RS_INF;
    float best32 = __builtin_huge_valf();
    int bp = -1;
    int node = S.root;
    int sp = 0;
#ifdef RS_TRAV_STATS
    int st_nodes = 0, st_leaves = 0, st_witer = 0;
#define RS_ST_NODE() ++st_nodes
#define RS_ST_LEAF() ++st_leaves
#else
#define RS_ST_NODE()
#define RS_ST_LEAF()
#endif
// a leaf: child code ~e names leaf entry e (rs_layout.h)
#define RS_LEAF(code)                                                          \
    do {                                                                       \
        RS_ST_LEAF();                                                          \
        const int bp_prev = bp;                                                \
        test_leaf<SM, LOBJ>(S, ~(code), r, rc, tmin, best, bend, bp);          \
        if (bp != bp_prev || bp >= 0) best32 = round_up_f(best);               \
    } while (0)
    // (the generic mode carries it too: its kernels include the World::hit probe, k_probe_hit, which
    // serves every scene mode's trees)
    if ((SM == kSmNest0 || SM == kSmNest2 || SM == kSmGeneric) && S.root4 >= 0 && S.ref_order) {
        // BVH::hit's recursion order on the in-order 4-wide tree (rs_host.cpp collapse4_inorder): the
        // slots of a node left to right, each child's box tested when it is reached with the range the
        // slots before it left behind; entering an inner child pushes (node, next slot).
        int k = 0;
        node = S.root4;
        while (true) {
            const uint32_t nb = (uint32_t)node * (uint32_t)sizeof(DNode4) + 4u * (uint32_t)k;
            const int c = nld<LOBJ, int>(S.nodes4, nb + 96u);
            if (c == INT32_MIN) {  // slots are filled from the left: the node is done
                if (sp == 0) break;
                --sp;
                const int v = stk.get(sp);
                node = v >> 2; k = v & 3;
                continue;
            }
            const float lo[3] = {nld<LOBJ, float>(S.nodes4, nb), nld<LOBJ, float>(S.nodes4, nb + 16u),
                                 nld<LOBJ, float>(S.nodes4, nb + 32u)};
            const float hi[3] = {nld<LOBJ, float>(S.nodes4, nb + 48u), nld<LOBJ, float>(S.nodes4, nb + 64u),
                                 nld<LOBJ, float>(S.nodes4, nb + 80u)};
            float e;
            if (slab32(lo, hi, rf, tmin32, best32, e)) {
                RS_ST_NODE();
                if (c < 0) {
                    RS_LEAF(c);
                } else {
                    if (k < 3) { stk.put(sp, node * 4 + k + 1); ++sp; }  // come back for the next slot
                    node = c;
                    k = 0;
                    continue;
                }
            }
            if (k < 3) { ++k; continue; }
            if (sp == 0) break;
            --sp;
            const int v = stk.get(sp);
            node = v >> 2; k = v & 3;
        }
    } else if (S.root4 >= 0 && !S.ref_order) {
        // 4-wide near-first (bvh4_step): nearest inner child next, the rest pushed far-to-near
        const RayF4 rq = make_rayf4(rf);
        node = S.root4;
        while (node >= 0) {
            RS_ST_NODE();
            node = bvh4_step<SM, STK, LOBJ, TOP>(S, r, rc, rq, tmin, tmin32, node, sp, stk, best, bend, bp, best32 RS_ST_PASS);
        }
    } else {
        // (the generic mode's reference-order scenes: boxes / quadrics / CSG in rich scenes) BVH::hit's
        // recursion order (bvh.rs:173-192) on the binary tree, one child per pass: k = 0 the left child,
        // k = 1 the right one (its box tested with the range the left subtree left behind); an inner
        // left child is entered with the node pushed to come back for its right child. One leaf-test
        // site, so the nested-object tests are inlined once.
        int k = 0;
        while (true) {
            const DNode& N = S.nodes[node];
            const int c = N.child[k];
            float e;
            if (c != INT32_MIN && slab32(N.lo[k], N.hi[k], rf, tmin32, best32, e)) {
                if (c < 0) {
                    RS_LEAF(c);
                } else {
                    if (k == 0) { stk.put(sp, node); ++sp; }  // come back for the right child
                    node = c;
                    k = 0;
                    continue;
                }
            }
            if (k == 0) { k = 1; continue; }
            if (sp == 0) break;
            --sp;
            node = stk.get(sp);
            k = 1;
        }
    }
#undef RS_LEAF
#ifdef RS_TRAV_STATS
    s_st_nodes[threadIdx.x] = st_nodes;   // reduced per wave by the kernel (rs_trav_stats_flush)
    s_st_leaves[threadIdx.x] = st_leaves;
    s_st_witer[threadIdx.x] = st_witer;
#endif
    bend_out = TOUT ? best : bend;
    return (bp >= 0 && S.lprim) ? S.lprim[bp] : bp;
}

// The record of a leaf object or of a TfFacade chain over one (tf_facade.rs:41-55): Obj::hit without
// the CSG code. The material classes 0-3 hold only such prims (rs_host.cpp class_of: composites are
// class 4), so their shading batches take this smaller finish.
template <int L>
__device__ __forceinline__ bool leafish_hit(const DScene& S, int pi, const Ray& r, double tmin, double tmax, Hit& h) {
    if constexpr (L > 0) {
        const DPrim P = S.prims[pi];
        if (P.kind == PK_XFORM) {
            const DXform X = S.xforms[P.idx];
            Ray rr = r;
            rr.o = r.o; rr.d = r.d;
            tf_inverse_ray(S, X, P.aux, rr.o, rr.d);
            if (!leafish_hit<L - 1>(S, X.child, rr, tmin, tmax, h)) return false;
            h.p = tf_forward(S, X, P.aux, h.p, 1.0);
            return true;
        }
    }
    return Obj<0, 0>::hit(S, pi, r, tmin, tmax, h);
}

// Recompute the full record of the winner with the exact range it was accepted under. LEAFISH: the
// prim is a leaf or a TfFacade chain over one (leafish_hit).
template <int SM, bool LEAFISH = false>
__device__ __forceinline__ bool finish_hit(const DScene& S, int bp, const Ray& r, double tmin, double bend, Hit& h) {
    if (bp < 0) return false;
    if constexpr (LEAFISH && (SM == kSmNest0 || SM == kSmNest2)) return leafish_hit<nest_of(SM)>(S, bp, r, tmin, bend, h);
    if ((SM == kSmSpheres) || S.prims[bp].kind == PK_SPHERE) {
        const DPrim P = S.prims[bp];
        return sphere_hit(S.spheres[P.idx], P.mat, r, tmin, bend, h, rich_of(SM) ? S.uv : 0);
    }
    if (SM == kSmFlat) return flat_hit(S, S.prims[bp], r, tmin, bend, h);
    return obj_hit<SM>(S, bp, r, tmin, bend, h);
}

template <int SM, class STK>
__device__ __forceinline__ bool world_hit(const DScene& S, const Ray& r, double tmin, Hit& h, const STK& stk) {
    double bend;
    const int bp = traverse<SM>(S, r, tmin, bend, stk);
    return finish_hit<SM>(S, bp, r, tmin, bend, h);
}

// camera.rs:94-100
__device__ __forceinline__ double phong_highlight(V3 dir_to_light, V3 ray_dir, V3 n, int exponent, double factor) {
    V3 reflected = dir_to_light - (2.0 * dot(dir_to_light, n)) * n;
    double spec = powi_rt(fmax(dot(reflected, -ray_dir), 0.0), exponent);
    return spec * factor;
}

// Scatter on a surface material (after MixedMaterial resolution) and the non-skip_pdf sampling
// of camera.rs:176-247. KIND is the material class when known at compile time (material-sorted
// wavefront shading) or -1 for a runtime switch. M0 = the hit's material (settings() source),
// M = the material that scatters. Returns true when the path continues; *light_ray (when given)
// is set to 1 if the next ray is a light sample.
template <int KIND, int SM>
__device__ __forceinline__ bool shade_surface(const DScene& S, const Hit& h, const DMaterial& M0, const DMaterial& M,
                                              Ray& ray, V3& T, Rng& rng, int* light_ray = nullptr) {
    const int kind = KIND >= 0 ? KIND : M.kind;
    float c[3];
    Pdf pdf;
    if (kind == RS_MAT_METAL) {  // metal.rs:104-118
        tex_color<rich_of(SM)>(S, M, h, c);
        V3 rf = reflect_v(ray.d, h.n);
        if (!(dot(rf, h.n) > 0.0)) return false;
        T = v3(T.x * (double)c[0], T.y * (double)c[1], T.z * (double)c[2]);
        ray.o = h.p; ray.d = rf;
        return true;
    } else if (kind == RS_MAT_DIELECTRIC) {  // dielectric.rs:55-93
        V3 nd;
        double cos_theta = dot(-ray.d, h.n);
        double sin_theta = sqrt(1.0 - cos_theta * cos_theta);
        double refr = h.outside ? M.enter_refractive : M.outer_refractive;
        bool refracted = false;
        if (!(refr * sin_theta > 1.0)) {
            double reflect_prob = 0.0;
            if (M.glass) {  // Glass::reflect_prob, powi(5) = x * ((x*x)*(x*x))
                double r0 = (1.0 - refr) / (1.0 + refr);
                r0 = r0 * r0;
                double x = 1.0 - cos_theta;
                double x2 = x * x;
                reflect_prob = fma(1.0 - r0, x * (x2 * x2), r0);
            }
            if (!(rng.gen() < reflect_prob)) {
                V3 rp = (ray.d + cos_theta * h.n) * refr;
                V3 rq = (-sqrt(1.0 - len2(rp))) * h.n;
                nd = rp + rq;
                refracted = true;
            }
        }
        if (!refracted) nd = reflect_v(ray.d, h.n);
        T = v3(T.x * (double)M.even[0], T.y * (double)M.even[1], T.z * (double)M.even[2]);
        ray.o = h.p; ray.d = nd;
        return true;
    } else if (kind == RS_MAT_LAMBERTIAN) {  // lambertian.rs:39-50
        tex_color<rich_of(SM)>(S, M, h, c);
        pdf.kind = kPdfCosine;
        pdf.n = onb_from(h.n);
    } else if (kind == RS_MAT_DIFFUSE_METAL) {  // metal.rs:54-68
        tex_color<rich_of(SM)>(S, M, h, c);
        V3 rf = reflect_v(ray.d, h.n);
        if (!(dot(rf, h.n) > 0.0)) return false;
        pdf.kind = kPdfReflection;
        pdf.exponent = M.exponent;
        pdf.refl = onb_from(rf);
        pdf.n = onb_from(h.n);
    } else if (rich_of(SM) && kind == RS_MAT_ISOTROPIC) {  // isotropic.rs:25-33
        c[0] = M.even[0]; c[1] = M.even[1]; c[2] = M.even[2];
        pdf.kind = kPdfSphere;
    } else if (rich_of(SM) && kind == RS_MAT_BLINN_PHONG) {  // blinn_phong.rs:32-42 + BlinnPhongPdf::new (pdf.rs:153-172)
        tex_color<rich_of(SM)>(S, M, h, c);
        pdf.kind = kPdfBlinnPhong;
        pdf.rin = ray.d;
        pdf.exponent = M.exponent;
        pdf.k = M.k_specular;
        pdf.refl = onb_from(reflect_v(ray.d, h.n));
        pdf.n = onb_from(h.n);
    } else {
        return false;  // DiffuseLight reached through MixedMaterial: scatter None, no emission
    }
    // non-skip_pdf branch (camera.rs:194-247)
    double light_multi = 1.0, pdf_val;
    Ray nr;
    nr.time = ray.time;
    if (rng.gen() < 0.5) {
        if (light_ray) *light_ray = 1;
        pdf_val = 0.3183098861837907;
        const uint32_t li = rng.next_u32() % (uint32_t)S.n_lights;  // list.rs:49-52
        V3 rv;
        if (SM == kSmSpheres) rv = Obj<0, 0>::sphere_random(S.spheres[S.prims[S.lights[li]].idx], h.p, rng);
        else if (SM == kSmFlat) rv = Obj<0, 0>::random(S, S.lights[li], h.p, rng);  // no nesting below a leaf
        else rv = obj_random<SM>(S, S.lights[li], h.p, rng);
        V3 dl = unit(rv);
        if (M0.phong_factor > 0.0) light_multi += phong_highlight(-dl, ray.d, h.n, M0.phong_exponent, M0.phong_factor);
        nr.o = ray_at(ray, h.t1 - 0.0002);
        nr.d = dl;
    } else {
        V3 sd = (KIND == RS_MAT_LAMBERTIAN) ? onb_local(pdf.n, random_cosine_direction(rng))
                                            : pdf_generate<rich_of(SM)>(pdf, rng);
        pdf_val = pdf_value<rich_of(SM)>(pdf, sd);
        nr.o = h.p;
        nr.d = sd;
    }
    if (pdf_val <= 0.0 || pdf_val != pdf_val) pdf_val = 1e-5;
    const double mult = pdf_value<rich_of(SM)>(pdf, nr.d) / pdf_val;
    T = v3(((double)c[0] * (light_multi * T.x)) * mult, ((double)c[1] * (light_multi * T.y)) * mult,
           ((double)c[2] * (light_multi * T.z)) * mult);
    ray = nr;
    return true;
}

// A path that ends without an emission term (absorbed: scatter None; or the depth limit, where
// ray_color returns 0) still multiplies that 0 through every level's factor in the reference's
// recursion (camera.rs:241-247): (color * (light_multi * 0)) * mult. In the forward form that is
// L + T * 0 -- which leaves L unchanged unless a factor was NaN / inf, where the recursion's
// result is NaN and so is this one.
__device__ __forceinline__ V3 close_path(V3 L, V3 T) { return L + T * 0.0; }

// DiffuseLight emission (light.rs:33-35) of the hit's material, as a radiance vector
template <int R>
__device__ __forceinline__ V3 emission(const DScene& S, const DMaterial& M0, const Hit& h) {
    float c[3];
    tex_color<R>(S, M0, h, c);
    return v3((double)c[0] * M0.multiplier, (double)c[1] * M0.multiplier, (double)c[2] * M0.multiplier);
}

// One level of TakePhotoSettings::ray_color (camera.rs:156-255) after world.hit: adds this
// level's contribution to L and, when the recursion continues, replaces `ray` and multiplies the
// path throughput T by this level's factor. Returns true when the path continues.
// KIND = RS_MAT_LAMBERTIAN: the scene's hits carry Lambertian or DiffuseLight materials only (DScene::lamb_only),
// so no MixedMaterial resolution and the Lambertian scatter alone
template <int SM, int KIND = -1>
__device__ bool shade_step(const DScene& S, bool hit_ok, const Hit& h, Ray& ray, V3& T, V3& L, Rng& rng) {
    if (!hit_ok) {  // camera.rs:253-254 background
        V3 bg = background(S, ray);
        L = L + v3(T.x * bg.x, T.y * bg.y, T.z * bg.z);
        return false;
    }
    const int mi = h.mat >= 0 ? h.mat : S.default_mat;
    const DMaterial& M0 = S.mats[mi];
    if (M0.kind == RS_MAT_DIFFUSE_LIGHT) {  // scatter None -> emitted
        V3 e = emission<rich_of(SM)>(S, M0, h);
        L = L + v3(T.x * e.x, T.y * e.y, T.z * e.z);
        return false;
    }
    if constexpr (KIND == RS_MAT_LAMBERTIAN) {
        if (shade_surface<RS_MAT_LAMBERTIAN, SM>(S, h, M0, M0, ray, T, rng)) return true;
        L = close_path(L, T);
        return false;
    }
    int ms = mi;
    for (int k = 0; k < 16 && S.mats[ms].kind == RS_MAT_MIXED; ++k) {  // mixed_material.rs:43-50
        const DMaterial& X = S.mats[ms];
        ms = ((double)rng.next_u32() < 4294967295.0 * X.mix_p) ? X.mix_a : X.mix_b;
    }
    if (shade_surface<-1, SM>(S, h, M0, S.mats[ms], ray, T, rng)) return true;
    L = close_path(L, T);  // scatter None
    return false;
}

// ray_color iterated: one world.hit per level, at most `depth` levels. Returns the radiance.
template <int SM>
__device__ V3 trace_path(const DScene& S, Ray ray, uint32_t depth, Rng& rng, const Stk& stk, uint32_t& segs) {
    V3 T = v3(1.0, 1.0, 1.0);
    V3 L = v3(0.0, 0.0, 0.0);
    for (uint32_t d = depth; d > 0; --d) {
        ++segs;
        Hit h;
        if (rich_of(SM) && S.has_media) ray.key = rng.medium_key();
        const bool ok = world_hit<SM>(S, ray, 0.0001, h, stk);
        if (!shade_step<SM>(S, ok, h, ray, T, L, rng)) return L;
    }
    return close_path(L, T);  // depth limit: the next level would return 0
}

template <int SM>
__global__ __launch_bounds__(kBlock) void k_path_mega(const DScene* __restrict__ Sp, DCamera C, PathParams P, double* __restrict__ rad,
                                                      unsigned long long* __restrict__ seg_counters) {
    const DScene& S = *Sp;  // the scene lives in device memory: no by-value copy in scratch
    __shared__ int stk_all[kStackMax * kBlock];
    const Stk stk = make_stk(S, stk_all);
    uint32_t segs = 0;
    // grid-stride (the host bounds the grid, which also bounds the stack overflow array)
    for (uint64_t item = (uint64_t)blockIdx.x * kBlock + threadIdx.x; item < P.n_items;
         item += (uint64_t)gridDim.x * kBlock) {
        const uint32_t pl = (uint32_t)(item % P.n_pix_local);
        const uint32_t sl = (uint32_t)(item / P.n_pix_local);
        const uint32_t x = pl % P.width;
        const uint32_t y = P.row_begin + (pl / P.width) * P.row_step;
        const uint64_t pix = (uint64_t)y * P.width + x;
        V3 L = v3(0.0, 0.0, 0.0);
        if (!P.mask || P.mask[pix]) {
            const uint32_t s = P.s0 + sl;
            Rng rng;
            rng.seed_from_u64(splitmix64(splitmix64(P.key_base ^ pix) ^ (uint64_t)s));
            const uint32_t si = s % P.sqrt_spp, sj = s / P.sqrt_spp;
            // painter.rs:167-170 (x draw first) + calculate_uv painter.rs:133-139
            const double sq = (double)P.sqrt_spp;
            const double xo = (double)x + ((double)si + rng.gen()) / sq;
            const double yo = (double)y + ((double)sj + rng.gen()) / sq;
            const double hh = (double)P.height;
            const double u = xo / (double)P.width;
            const double v = (hh - 1.0 - yo) / hh;
            Ray r = camera_ray(C, u, v, rng);
            L = trace_path<SM>(S, r, P.depth, rng, stk, segs);
        }
        put_rad(rad, item, L.x, L.y, L.z);
    }
    // wave-reduce the segment count, one atomic per wave, spread over 256 counters
    unsigned long long s64 = segs;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s64 += __shfl_xor(s64, off, 64);
    if ((threadIdx.x & 63) == 0 && s64) atomicAdd(&seg_counters[blockIdx.x & 255], s64);
}

// ============================================================== wavefront path ====
// Path state is SoA-of-32-byte-records in HBM (one record per array per path, so a wave's
// load is 2 KiB contiguous). Bounce b: k_wf_extend traverses every path on queue b and writes
// (prim, range end); k_wf_shade finishes the record, applies the material and appends the
// surviving paths to queue b+1 with one atomic per wave (ballot + popcount prefix).
// path records (rs_internal.h WfSet): two rng words as the bits of one double, never computed with
__device__ __forceinline__ double pack_u32x2(uint32_t lo, uint32_t hi) {
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ void unpack_u32x2(double v, uint32_t& lo, uint32_t& hi) {
    const uint64_t u = (uint64_t)__double_as_longlong(v);
    lo = (uint32_t)u;
    hi = (uint32_t)(u >> 32);
}
// tw (WfState::tagw): the scene has no moving sphere, so a path's time is never read (a static sphere's centre
// is c + 0 * t = c for any finite t >= 0, sphere.rs center_at), and its record carries (item, level) in ray_o.w
// instead of the tag array: 8 B less each way per record (the shading is bound by its record traffic)
__device__ __forceinline__ Ray load_ray(const WfSet& W, uint32_t p, bool tw = false, uint2* tag = nullptr) {
    const D4 a = W.ray_o[p], b = W.ray_d[p];
    Ray r;
    r.o = v3(a.x, a.y, a.z); r.time = tw ? 0.0 : a.w;
    r.d = v3(b.x, b.y, b.z);
    r.key = 0;
    if (tag) {
        if (tw) unpack_u32x2(a.w, tag->x, tag->y);
        else *tag = W.tag[p];
    }
    return r;
}
__device__ __forceinline__ Rng load_rng(const WfSet& W, uint32_t p) {
    Rng g;
    unpack_u32x2(W.ray_d[p].w, g.x, g.y);
    unpack_u32x2(W.thr[p].w, g.z, g.w);
    return g;
}
__device__ __forceinline__ void load_path(const WfSet& W, uint32_t p, Ray& r, V3& T, Rng& rng, bool tw, uint2& tag) {
    const D4 a = W.ray_o[p], b = W.ray_d[p], t = W.thr[p];
    r.o = v3(a.x, a.y, a.z); r.time = tw ? 0.0 : a.w;
    r.d = v3(b.x, b.y, b.z);
    r.key = 0;
    T = v3(t.x, t.y, t.z);
    unpack_u32x2(b.w, rng.x, rng.y);
    unpack_u32x2(t.w, rng.z, rng.w);
    if (tw) unpack_u32x2(a.w, tag.x, tag.y);
    else tag = W.tag[p];
}
__device__ __forceinline__ void store_path(const WfSet& W, uint32_t p, const Ray& r, const V3& T, const Rng& rng,
                                           uint32_t item, uint32_t level, bool tw) {
    D4 a, b, t;
    a.x = r.o.x; a.y = r.o.y; a.z = r.o.z; a.w = tw ? pack_u32x2(item, level) : r.time;
    b.x = r.d.x; b.y = r.d.y; b.z = r.d.z; b.w = pack_u32x2(rng.x, rng.y);
    t.x = T.x; t.y = T.y; t.z = T.z; t.w = pack_u32x2(rng.z, rng.w);
    W.ray_o[p] = a; W.ray_d[p] = b; W.thr[p] = t;
    if (!tw) W.tag[p] = make_uint2(item, level);
}

// Block-aggregated slot allocation for up to C independent counters: ONE returning atomic per
// block and counter (a single hot word sustains only ~88 atomics/us, MI355X_MICROARCH.md
// 'dequeue'), lanes get slots ordered by (wave, lane). Must be called by every thread of the block.
// With stat != nullptr the block's count of `flag` lanes is also added to *stat (no returned value).
template <int C>
__device__ __forceinline__ uint32_t block_slot(int cls, uint32_t* const* counters, bool flag = false,
                                               uint32_t* stat = nullptr) {
    __shared__ uint32_t wcnt[C + 1][kBlock / 64];
    __shared__ uint32_t bbase[C];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned long long mine = 0ull;
#pragma unroll
    for (int k = 0; k < C; ++k) {
        const unsigned long long m = __ballot(cls == k);
        if (cls == k) mine = m;
        if (lane == 0) wcnt[k][wave] = (uint32_t)__popcll(m);
    }
    if (stat) {
        const unsigned long long m = __ballot(flag);
        if (lane == 0) wcnt[C][wave] = (uint32_t)__popcll(m);
    }
    __syncthreads();
    if (threadIdx.x < C) {
        const int k = threadIdx.x;
        uint32_t tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) { const uint32_t c = wcnt[k][w]; wcnt[k][w] = tot; tot += c; }
        bbase[k] = tot ? atomicAdd(counters[k], tot) : 0u;
    } else if (stat && threadIdx.x == 64) {
        uint32_t tot = 0;
        for (int w = 0; w < kBlock / 64; ++w) tot += wcnt[C][w];
        if (tot) atomicAdd(stat, tot);
    }
    __syncthreads();
    uint32_t slot = 0;
    if (cls >= 0 && cls < C) slot = bbase[cls] + wcnt[cls][wave] + (uint32_t)__popcll(mine & ((1ull << lane) - 1ull));
    __syncthreads();  // wcnt / bbase are reused by the next call
    return slot;
}
__device__ __forceinline__ uint32_t block_slot1(bool flag, uint32_t* counter) {
    uint32_t* const cs[1] = {counter};
    return block_slot<1>(flag ? 0 : -1, cs);
}

// painter.rs:167-170 + camera.rs:77-85 for every (pixel, sample) item of a chunk
// Camera sample `item` of the batch (painter.rs:154-187 jitter, camera.rs:77-85 ray): false for a
// masked pixel (painter.rs:204-210) or depth 0 (camera.rs:161), whose radiance is 0.
__device__ __forceinline__ void camera_sample_xy(const DCamera& C, const PathParams& P, uint64_t key, uint32_t x,
                                                 uint32_t y, uint32_t s, Ray& r, Rng& rng) {
    const uint64_t pix = (uint64_t)y * P.width + x;
    rng.seed_from_u64(splitmix64(splitmix64(key ^ pix) ^ (uint64_t)s));
    const uint32_t si = s % P.sqrt_spp, sj = s / P.sqrt_spp;
    const double sq = (double)P.sqrt_spp;
    const double xo = (double)x + ((double)si + rng.gen()) / sq;
    const double yo = (double)y + ((double)sj + rng.gen()) / sq;
    const double hh = (double)P.height;
    r = camera_ray(C, xo / (double)P.width, (hh - 1.0 - yo) / hh, rng);
}
__device__ __forceinline__ bool camera_sample(const DCamera& C, const PathParams& P, uint64_t key, uint64_t item, Ray& r,
                                              Rng& rng) {
    const uint32_t pl = (uint32_t)(item % P.n_pix_local);
    const uint32_t sl = (uint32_t)(item / P.n_pix_local);
    const uint32_t x = pl % P.width;
    const uint32_t y = P.row_begin + (pl / P.width) * P.row_step;
    const uint64_t pix = (uint64_t)y * P.width + x;
    if ((P.mask && !P.mask[pix]) || P.depth == 0) return false;
    camera_sample_xy(C, P, key, x, y, P.s0 + sl, r, rng);
    return true;
}
__device__ __forceinline__ bool camera_sample(const DCamera& C, const PathParams& P, uint64_t item, Ray& r, Rng& rng) {
    return camera_sample(C, P, P.key_base, item, r, rng);
}

// Camera-ray order: the i-th camera sample a launch traces is item gen_perm(i) of its batch (whole
// sample planes). A wave traces SP samples of each of 64 / SP lattice pixels: the batch's planes are cut into
// groups of RS_PIX_SAMPLES planes and the rest into groups of decreasing powers of two (15 planes: 8, 4, 2, 1),
// and inside a group of SP planes the i-th sample is plane i % SP of pixel i / SP in the pixels' tile order. The
// camera rays of one pixel differ by the sub-pixel jitter and the lens disk only, so a wave of one pixel's
// samples walks nearly one ray's nodes, and its hits, scattered rays and shading records stay together in the
// later iterations' queues. Against one sample plane per wave (round 6): 32 samples of 2 pixels per wave, bench
// frame 6.344 -> 6.212 ms, N = 8 share 0.900 -> 0.843 ms; 64 / 16 / 8 samples 6.260 / 6.226 / 6.232 ms; a C3-shaped
// frame 41.6 -> 40.8 ms; C4, C5, C2 and X1 shapes equal (profiles/r6/ab/pix_samples_r7c.txt, _scenes_r7c.jsonl).
// The pixels are visited in TW x TH tiles (TW * TH = 64 / SP; with one sample per pixel a 64 x 1 row strip spans
// 8x the angle of an 8 x 8 tile -- bench frame 10.21 -> 9.89 ms in round 2), the pixels outside the whole tiles
// after them in row-major order. Pure scheduling: rad[] is indexed by item, so the frame does not depend on it. A batch that is not whole planes keeps the identity order.
#ifndef RS_PIX_SAMPLES
#define RS_PIX_SAMPLES 32u
#endif
__device__ __forceinline__ uint32_t gen_perm(uint32_t i, uint64_t item0, uint32_t n, const PathParams& P) {
    const uint32_t npl = P.n_pix_local, W = P.width;
    if ((item0 % npl) != 0 || (n % npl) != 0) return i;
    constexpr uint32_t M = RS_PIX_SAMPLES;  // a power of two <= 64
    const uint32_t planes = n / npl, nfull = planes / M;
    uint32_t SP = M, p0, r;  // i's group: its planes, first plane, and i's index inside it
    if (i < nfull * M * npl) {
        const uint32_t g = i / (M * npl);
        p0 = g * M;
        r = i - g * (M * npl);
    } else {
        p0 = nfull * M;
        r = i - p0 * npl;
        uint32_t left = planes - p0;  // 1 .. M - 1
        SP = 1u << (31u - __clz(left));
        while (r >= SP * npl) {
            r -= SP * npl;
            p0 += SP;
            left -= SP;
            SP = 1u << (31u - __clz(left));
        }
    }
    const uint32_t TP = 64u / SP;  // pixels per wave
    // A lattice with row step k (a strong-scaled share: rows r, r + k, ...) puts TH lattice rows
    // TH * k screen rows apart: keep the tile near square on screen (64-pixel tiles: step >= 8: 16 x 4,
    // 4-7: 32 x 2, 2-3: 16 x 4; step 1: 8 x 8)
    uint32_t TH = 1u << ((31u - __clz(TP)) / 2);
#ifndef RS_SHARE_TH8
#define RS_SHARE_TH8 4u  // lattice rows per tile at row step >= 8 (16 x 4 lattice = 16 x 25 screen px at step 8; 64 x 1: N = 8 share 0.9416 -> 0.9313 ms, 32 x 2: 0.9342; profiles/r6/ab/variants_r6c_leaf2_th.txt)
#endif
    if (P.row_step > 1) TH = min(TH, P.row_step >= 8 ? RS_SHARE_TH8 : P.row_step >= 4 ? 2u : 4u);
    const uint32_t TW = TP / TH;
    const uint32_t s = p0 + r % SP;  // sample plane
    uint32_t q = r / SP, pl;         // the pixel's position in the tile order
    const uint32_t R = npl / W, Wt = W - W % TW, Rt = R - R % TH, nt = Wt * Rt;
    if (q < nt) {
        const uint32_t t = q / TP, k = q % TP, tpr = Wt / TW;
        const uint32_t ty = t / tpr, tx = t - ty * tpr;
        pl = (ty * TH + k / TW) * W + tx * TW + k % TW;
    } else {
        q -= nt;  // the right strip of the tiled rows, then the rows below
        const uint32_t rw = W - Wt;
        if (q < rw * Rt) {
            const uint32_t lr = q / rw;
            pl = lr * W + Wt + (q - lr * rw);
        } else {
            pl = Rt * W + (q - rw * Rt);
        }
    }
    return s * npl + pl;
}

// The camera sample behind the streaming iteration's injected record jg (0-based among its injections):
// its frame item g (camera_sample), its pass's key and its radiance slot in the rad ring.
__device__ __forceinline__ void inj_sample(const InjParams& I, const PathParams& P, uint32_t jg, uint64_t& g,
                                           uint64_t& key, uint32_t& item) {
    uint32_t jb = I.jb0 + jg, nb = I.nb0;
    uint64_t g0 = I.g0;
    item = I.rad0;
    key = I.key0;
    if (jb >= I.nb0) { jb -= I.nb0; nb = I.nb1; g0 = I.g1; item = I.rad1; key = I.key1; }
    const uint32_t perm = gen_perm(jb, 0, nb, P);
    item += perm;
    g = g0 + perm;
}

// k_wf_extend_dyn's chunk counters (WfState::fetch): zeroed by one thread of the launch before it
constexpr uint32_t kFetchCounters = 8, kFetchStride = 32;  // counters, words apart
__device__ __forceinline__ void zero_fetch(const WfState& W) {
    if (blockIdx.x == 0 && threadIdx.x < kFetchCounters) W.fetch[threadIdx.x * kFetchStride] = 0u;
}

// ---- sharded path sets of the bounce-synchronous wavefront ----
// A launch that compacts its survivors into the next set does it per block: one returning atomic per
// block on a count. On one word that saturates at ~88 atomics/us (MI355X_MICROARCH.md, 'dequeue') and its
// latency grows with the blocks waiting on it: with the mesh shading at 4 waves the bounce-0 launch took
// 2.54 ms, 1.56 ms with the same atomics spread over 8 words (profiles/r5/ab/c5_slot_spread_r5s.txt). So a
// set is kShards shards: input tile t (kBlock items of the producer's input, in its virtual order) sends
// its survivors to shard t % kShards, whose region has room for every item of its tiles (shard_cap); a
// shard's survivors are compacted at the start of its region. WfState::heads holds two banks (set b in bank
// b & 1) of kShards (count, region offset) pairs on their own 128-byte lines. A consumer walks the set in
// virtual order (shard 0's survivors, then shard 1's, ...: seg_pos). The extend of bounce b publishes the
// set's size in counts[b] (the host's statistics) and zeroes the other bank's counts for the shading of b.
constexpr uint32_t kShards = 8, kShardStride = 32;  // shards, words apart
__device__ __forceinline__ uint32_t* shard_bank(const WfState& W, uint32_t b) {
    return W.heads + (b & 1u) * (kShards * kShardStride);
}
struct Segs {
    uint32_t cnt[kShards], off[kShards];
    uint32_t n;
};
__device__ __forceinline__ Segs load_segs(const WfState& W, uint32_t b) {
    const uint32_t* h = shard_bank(W, b);
    Segs g;
    g.n = 0;
#pragma unroll
    for (uint32_t k = 0; k < kShards; ++k) {
        g.cnt[k] = h[k * kShardStride];
        g.off[k] = h[k * kShardStride + 1];
        g.n += g.cnt[k];
    }
    return g;
}
// virtual index v (< g.n) -> the record's position
__device__ __forceinline__ uint32_t seg_pos(const Segs& g, uint32_t v) {
    uint32_t pos = 0, pre = 0;
#pragma unroll
    for (uint32_t k = 0; k < kShards; ++k) {
        if (v >= pre && v - pre < g.cnt[k]) pos = g.off[k] + (v - pre);
        pre += g.cnt[k];
    }
    return pos;
}
// items of shard h's tiles for an input of n items (tile t = items [t * kBlock, (t + 1) * kBlock) -> shard t % kShards)
__device__ __forceinline__ uint32_t shard_cap(uint32_t n, uint32_t h) {
    const uint32_t F = n / kBlock, rem = n % kBlock;
    const uint32_t full = F > h ? (F - h + kShards - 1) / kShards : 0u;
    return full * kBlock + (F % kShards == h ? rem : 0u);
}
__device__ __forceinline__ uint32_t shard_off(uint32_t n, uint32_t h) {
    uint32_t o = 0;
    for (uint32_t j = 0; j < h; ++j) o += shard_cap(n, j);
    return o;
}
// the producer of bank b's set, input of n items: the shards' region offsets (block 0)
__device__ __forceinline__ void publish_offsets(const WfState& W, uint32_t b, uint32_t n) {
    if (blockIdx.x == 0 && threadIdx.x < kShards) shard_bank(W, b)[threadIdx.x * kShardStride + 1] = shard_off(n, threadIdx.x);
}
// the consumer of set b (the extend): its size for the host, and the other bank's counts zeroed for the
// shading's survivors (that bank's set, b - 1, is done with)
__device__ __forceinline__ void extend_prologue(const WfState& W, uint32_t b, uint32_t n) {
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) W.counts[b] = n;
        if (threadIdx.x < kShards) shard_bank(W, b + 1)[threadIdx.x * kShardStride] = 0u;
    }
}

#if RS_TU_COMMON
// The chunk's camera samples (set 0). Without a pixel mask every sample is live and record i is item i
// (one shard holding all n); with one, the live samples are compacted into shards (counts zeroed by the host).
__global__ __launch_bounds__(kBlock) void k_wf_gen(DCamera C, PathParams P, WfState W, uint64_t item0, uint32_t n,
                                                   double* __restrict__ rad) {
    zero_fetch(W);
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    bool live = false;
    Ray r;
    Rng rng;
    uint64_t item = 0;
    if (i < n) {
        item = item0 + gen_perm(i, item0, n, P);
        live = camera_sample(C, P, item, r, rng);
        if (!live) put_rad(rad, item, 0.0, 0.0, 0.0);
    }
    if (!P.mask && P.depth > 0) {
        // eight contiguous shards of whole 64-record chunks (the extend's waves draw from all eight counters)
        if (blockIdx.x == 0 && threadIdx.x < kShards) {
            uint32_t* const h = shard_bank(W, 0) + threadIdx.x * kShardStride;
            const uint32_t step = ((n + kShards - 1) / kShards + 63u) & ~63u;
            const uint32_t a = min(n, threadIdx.x * step), b = min(n, a + step);
            h[0] = b - a;
            h[1] = a;
        }
        if (live) store_path(W.set[0], i, r, v3(1.0, 1.0, 1.0), rng, (uint32_t)item, 0u, W.tagw);
        return;
    }
    publish_offsets(W, 0, n);
    const uint32_t sh = blockIdx.x % kShards;
    const uint32_t slot = block_slot1(live, shard_bank(W, 0) + sh * kShardStride);
    if (live) store_path(W.set[0], shard_off(n, sh) + slot, r, v3(1.0, 1.0, 1.0), rng, (uint32_t)item, 0u, W.tagw);
}
#endif  // RS_TU_COMMON

// flat scenes (meshes) are traversal-latency bound: their extend keeps 5 waves/SIMD (98 -> 96 VGPRs;
// unbounded, the mesh frame lost 18 %)
constexpr int kWfExtFlatWaves = 5;
template <int SM>
__global__ __launch_bounds__(kBlock, SM == kSmFlat ? kWfExtFlatWaves : 1) void k_wf_extend(const DScene* __restrict__ Sp, WfState W, uint32_t bounce) {
    const DScene& S = *Sp;  // the scene lives in device memory: no by-value copy in scratch
    __shared__ int stk_all[stack_lds(SM) * kBlock];
    const StkT<true, stack_lds(SM)> stk = make_stk<true, stack_lds(SM)>(S, stk_all);
    __shared__ int leafq[SM == kSmFlat ? RS_LEAFQ * kBlock : 1];
    const Segs in = load_segs(W, bounce);
    const uint32_t n = in.n;
    extend_prologue(W, bounce, n);
    const WfSet& cur = W.set[bounce & 1];
    for (uint32_t base = blockIdx.x * kBlock; base < n; base += gridDim.x * kBlock) {
        const uint32_t v = base + threadIdx.x;
        if (v < n) {
            const uint32_t i = seg_pos(in, v);
            Ray r = load_ray(cur, i, W.tagw);
            if (rich_of(SM) && S.has_media) r.key = load_rng(cur, i).medium_key();  // the segment's medium key
            double bend = RS_INF;
            int bp;
            if (SM == kSmFlat && S.root4 >= 0)
                bp = traverse_flat_q<SM>(S, r, 0.0001, bend, stk, leafq + threadIdx.x);
            else
                bp = traverse<SM>(S, r, 0.0001, bend, stk);
            W.hit[i] = make_double2(__longlong_as_double((long long)bp), bend);
        }
#ifdef RS_TRAV_STATS
        trav_stats_flush(v < n);
#endif
    }
}

// Flat scenes (meshes), persistent extend with lane refill. In k_wf_extend a wave lives as long as its
// slowest lane: on the C5 mesh a ray takes 18.6 node steps on average against a wave maximum of 41 (lane
// efficiency 0.45, profiles/r5/iters/trav_stats_r5c.txt). Here a lane whose ray is done takes the next
// one. A wave draws chunks of 64 records of one shard of the set from that shard's counter (W.fetch, 128 B
// apart; the wave starts on shard blockIdx % 8 -- one per XCD under round-robin dispatch, a speed choice
// only -- and moves to the next shard when its shard is empty), and refills its idle lanes from its pool
// of drawn records once RS_REFILL of them are idle (C5-shaped frame, extend per frame: 16 -> 83.8 ms,
// 32 -> 82.1, 48 +2 %, one ray per lane (k_wf_extend) 97.2; profiles/r5/ab/c5_dyn_r5*.jsonl). Each ray's
// walk is traverse_flat_q's (the same passes, a lane's own leaf FIFO and stack column), so its hit does
// not depend on its lane, wave or refill time. The counters are zeroed by the launch before (k_wf_gen,
// k_wf_shade) on the same stream.
#ifndef RS_REFILL
#define RS_REFILL 32
#endif
template <int SM>
__global__ __launch_bounds__(kBlock, kWfExtFlatWaves) void k_wf_extend_dyn(const DScene* __restrict__ Sp, WfState W,
                                                                            uint32_t bounce) {
    const DScene& S = *Sp;
    __shared__ int stk_all[stack_lds(SM) * kBlock];
    const StkT<true, stack_lds(SM)> stk = make_stk<true, stack_lds(SM)>(S, stk_all);
    __shared__ int leafq[RS_LEAFQ * kBlock];
    int* const q = leafq + threadIdx.x;
    const Segs in = load_segs(W, bounce);
    extend_prologue(W, bounce, in.n);
    const WfSet& cur = W.set[bounce & 1];
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t below = (1ull << lane) - 1ull;
    constexpr double tmin = 0.0001;
    const float tmin32 = -round_up_f(-tmin);
    // the wave's pool of drawn records [pa, pa + pn) (wave-uniform), its shard, shards found empty
    uint32_t pa = 0, pn = 0;
    uint32_t ck = blockIdx.x % kFetchCounters, tries = 0;
    int i = -1, bp = -1, node = -1, sp = 0, qh = 0, qt = 0;
    Ray r;
    r.o = r.d = v3(0.0, 0.0, 0.0);
    r.time = 0.0;
    RayF4 rq = make_rayf4(make_rayf(r.o, r.o));
    double best = RS_INF, bend = RS_INF;
    float best32 = __builtin_huge_valf();
    while (true) {
        const bool idle = node < 0 && qt == qh;
        if (idle && i >= 0) {
            W.hit[i] = make_double2(__longlong_as_double((long long)((bp >= 0 && S.lprim) ? S.lprim[bp] : bp)), bend);
            i = -1;
        }
        const uint64_t im = __ballot(idle);
        const uint32_t ni = (uint32_t)__popcll(im);
        if (ni >= RS_REFILL && (pn > 0 || tries < kFetchCounters)) {
            uint32_t pb = 0, pbn = 0;  // a chunk drawn when the pool cannot serve every idle lane
            while (pn < ni && tries < kFetchCounters) {
                uint32_t cnt = 0, off = 0;
#pragma unroll
                for (uint32_t k = 0; k < kShards; ++k)
                    if (k == ck) { cnt = in.cnt[k]; off = in.off[k]; }
                if (cnt > 0) {
                    uint32_t c = 0;
                    if (lane == 0) c = atomicAdd(W.fetch + ck * kFetchStride, 1u);
                    c = (uint32_t)__shfl((int)c, 0) * 64u;
                    if (c < cnt) { pb = off + c; pbn = min(64u, cnt - c); break; }
                }
                ck = (ck + 1) % kFetchCounters;
                ++tries;
            }
            if (idle) {
                const uint32_t k = (uint32_t)__popcll(im & below);
                uint32_t j = UINT32_MAX;
                if (k < pn) j = pa + k;
                else if (k - pn < pbn) j = pb + (k - pn);
                if (j != UINT32_MAX) {
                    i = (int)j;
                    r = load_ray(cur, j, W.tagw);
                    rq = make_rayf4(make_rayf(r.o, v3(1.0 / r.d.x, 1.0 / r.d.y, 1.0 / r.d.z)));
                    best = RS_INF; bend = RS_INF; best32 = __builtin_huge_valf();
                    bp = -1; node = S.root4; sp = 0; qh = 0; qt = 0;
                }
            }
            if (ni <= pn) { pa += ni; pn -= ni; }
            else { const uint32_t u = min(ni - pn, pbn); pa = pb + u; pn = pbn - u; }
        }
        const bool has_leaf = qt != qh;
        const bool can_node = node >= 0 && qt - qh <= RS_LEAFQ - 4;
        const uint64_t work = __ballot(node >= 0 || has_leaf);
        if (work == 0ull) break;  // every lane idle after a refill attempt: pool and shards are empty
        const uint64_t lm = __ballot(has_leaf);
        if (__popcll(lm) * 64 >= RS_LEAFQ_THR * __popcll(work) || __ballot(can_node) == 0ull) {
            if (has_leaf) {
                const int code = q[(qh & (RS_LEAFQ - 1)) * kBlock];
                ++qh;
                const int bp_prev = bp;
                test_leaf<SM>(S, ~code, r, ray_consts(r), tmin, best, bend, bp);
                if (bp != bp_prev || bp >= 0) best32 = round_up_f(best);
            }
        } else if (can_node) {
            node = bvh4_node_q<SM>(S, rq, tmin32, best32, node, sp, stk, q, qt);
        }
    }
}

// LAMB: the scene's shading is Lambertian / DiffuseLight only (DScene::lamb_only), compiled for that alone
// (C5-shaped frame, shading per frame: 18.6 ms unbounded (3 waves), 22.4 at 4 waves (36 B of scratch), the
// generic kernel 23.5; profiles/r5/ab/c5_shards_r5t.txt)
#ifndef RS_LAMB_WAVES
#define RS_LAMB_WAVES 1
#endif
template <int SM, bool LAMB = false>
__global__ __launch_bounds__(kBlock, LAMB ? RS_LAMB_WAVES : 1) void k_wf_shade(const DScene* __restrict__ Sp, WfState W, uint32_t bounce, uint32_t depth,
                                                    uint64_t n_items, double* __restrict__ rad) {
    const DScene& S = *Sp;  // the scene lives in device memory: no by-value copy in scratch
    zero_fetch(W);          // for the next bounce's extend (this bounce's is done: same stream)
    const Segs in = load_segs(W, bounce);
    const uint32_t n = in.n;
    publish_offsets(W, bounce + 1, n);
    uint32_t* const out = shard_bank(W, bounce + 1);
    const WfSet& cur = W.set[bounce & 1];
    const WfSet& nxt = W.set[(bounce + 1) & 1];
    for (uint32_t base = blockIdx.x * kBlock; base < n; base += gridDim.x * kBlock) {
        const uint32_t v = base + threadIdx.x;
        bool alive = false;
        Ray r;
        V3 T, L = v3(0.0, 0.0, 0.0);  // a live path's radiance (WfSet)
        Rng rng;
        uint32_t item = 0;
        if (v < n) {
            const uint32_t i = seg_pos(in, v);
            uint2 tg;
            load_path(cur, i, r, T, rng, W.tagw, tg);
            if (rich_of(SM) && S.has_media) r.key = rng.medium_key();
            const double2 hb = W.hit[i];
            const int bp = (int)__double_as_longlong(hb.x);
            Hit h;
            const bool ok = finish_hit<SM>(S, bp, r, 0.0001, hb.y, h);
            item = tg.x;
            alive = shade_step<SM, LAMB ? RS_MAT_LAMBERTIAN : -1>(S, ok, h, r, T, L, rng);
            if (alive && bounce + 1 >= depth) {  // depth limit
                L = close_path(L, T);
                alive = false;
            }
            if (!alive) put_rad(rad, item, L.x, L.y, L.z);
        }
        const uint32_t sh = (base / kBlock) % kShards;
        const uint32_t slot = block_slot1(alive, out + sh * kShardStride);
        if (alive) store_path(nxt, shard_off(n, sh) + slot, r, T, rng, item, 0u, W.tagw);
    }
}

// ---- streaming material-sorted wavefront (spheres / nest-0 / nest-2 scenes) ----
// A frame is one sequence of iterations over a pool of paths in flight. Iteration t:
//  k_wfs_extend     World::hit for every path carried in from iteration t-1 (set t&1: light-sample
//                   rays from the front, the rest from the back) and for the camera samples injected
//                   at t, generated in the kernel (painter.rs:154-187, camera.rs:77-85). Sky misses and
//                   light hits end here (their radiance is written); the rest go to the queue of their
//                   material class.
//  k_wfs_shade_all  every class queue in one launch: scatter (camera.rs:176-250); the survivors are
//                   compacted into set (t+1)&1.
// The host injects a fixed number of camera samples per iteration, so the schedule needs no read-back:
// a sample injected at t traces its ray_color level b at iteration t + b and has finished by
// t + depth - 1, after which its batch's radiance may be accumulated. Paths of different levels share
// a launch; a record carries its level (WfSet::tag) for the depth limit. Every launch stays full until
// the frame's last samples are injected: no per-bounce tail of small launches per chunk.
// Class of a hit: a per-prim byte (DScene::pclass) computed at commit, k = 0 Lambertian, 1 Metal,
// 2 DiffuseMetal, 3 Dielectric, 4 other / MixedMaterial / composite; kClsLight marks DiffuseLight prims,
// whose paths end inside extend like sky misses (no queue, no second gather of the path state).
constexpr int kClasses = kWfsClasses;
constexpr int kClsLight = 6;

// waves/SIMD the extend is bounded to: spheres and nest-0 scenes 4 (128 VGPRs; the spheres-mode
// camera-ray extend 144 -> 128 VGPRs: bench frame 7.86 -> 7.63 ms; nest-0 129 -> 128: example.sdl
// 10.8 -> 10.3 ms; 5 waves spills and measured slower); nest-2 with the LDS image 3 (168 VGPRs, 184 B
// of scratch: 4 % faster than 2 waves, 4 waves 12 % slower; profiles/r4/ab/nest2_registers; round 5 on the
// C4-shaped frame: 2 waves 5.43 -> 4.54 Gseg/s, profiles/r5/ab/c4_waves_r5l), nest-2
// with its tables in global memory 2 (its loads are L1 / L2 round trips that the spills would join)
// The spheres mode's carried-path part (the divergent bounce >= 1 rays: lane efficiency 0.51 for BSDF rays,
// profiles/r5/iters) at 5 waves: 96 VGPRs, 12 B of scratch, 5 blocks of 24 KiB stacks per CU; bench frame
// 7.58 -> 7.31 ms. Its camera part keeps 4 (13 VGPRs would spill).
constexpr int ext_min_waves(int sm, bool lobj = false, int part = kExtAll) {
    if (sm == kSmSpheres && part == kExtCarried) return 5;
    // (the spheres camera part at 5 waves spills 108 B: bench frame +4 %, profiles/r6/ab/waves_cam_lean_r7i.txt)
    return sm == kSmNest2 ? (lobj ? 3 : 2) : 4;
}

// The scene's LDS image (DScene::limg, nest modes): the block copies it into its dynamic LDS and
// reads the tree and the object tables through a DScene copy whose table pointers point there.
// The copy is a by-value aggregate used only by inlined code, so it stays in SGPRs, and the
// compiler sees the tables' LDS origin (ds_read). The node -> prim -> CSG -> child -> shape
// chain of a nested-object test becomes LDS round trips instead of L1 / L2 ones.
extern __shared__ uint4 s_limg[];
// fill the block's copy of the image; every thread of the block calls it (barrier)
__device__ __forceinline__ void lds_fill(const DScene& Sv) {
    const uint32_t nq = Sv.limg_bytes >> 4;
    const uint4* __restrict__ src = (const uint4*)Sv.limg;
    for (uint32_t q = threadIdx.x; q < nq; q += kBlock) s_limg[q] = src[q];
    __syncthreads();
}
// Sv := the scene with its table pointers into the LDS copy (fill: also fill the copy)
__device__ __forceinline__ void lds_scene(const DScene* __restrict__ Sp, DScene& Sv, bool fill = true) {
    Sv = *Sp;
    if (fill) lds_fill(Sv);
    const char* b = (const char*)s_limg;
    Sv.nodes4 = (const DNode4*)(b + Sv.limg_off[LT_NODES4]);
    Sv.pclass = (const uint8_t*)(b + Sv.limg_off[LT_PCLASS]);
    Sv.pbox = (const DBox64*)(b + Sv.limg_off[LT_PBOX]);
    Sv.prims = (const DPrim*)(b + Sv.limg_off[LT_PRIMS]);
    Sv.spheres = (const DSphere*)(b + Sv.limg_off[LT_SPHERES]);
    Sv.rects = (const DRect*)(b + Sv.limg_off[LT_RECTS]);
    Sv.boxes = (const DBox*)(b + Sv.limg_off[LT_BOXES]);
    Sv.quadrics = (const DQuadric*)(b + Sv.limg_off[LT_QUADRICS]);
    Sv.csgs = (const DCsg*)(b + Sv.limg_off[LT_CSGS]);
    Sv.xforms = (const DXform*)(b + Sv.limg_off[LT_XFORMS]);
    Sv.tf_fwd = (const DMat34*)(b + Sv.limg_off[LT_TF_FWD]);
    Sv.tf_inv = (const DMat34*)(b + Sv.limg_off[LT_TF_INV]);
}
// PART (rs_internal.h): kExtAll -- the carried paths and the injected camera samples in one launch;
// kExtCarried / kExtCamera -- one of the two (an iteration then takes two launches): where the merged
// kernel needs more registers than either alone (nest-2: 256 VGPRs + 2 AGPRs, one wave per SIMD,
// against two waves for each part)
// LOBJ: the scene's tables from its LDS image (lds_scene; the launch passes limg_bytes of dynamic LDS)
template <int SM, bool OVF, int PART, bool LOBJ>
__global__ __launch_bounds__(kBlock, ext_min_waves(SM, LOBJ, PART)) void k_wfs_extend(const DScene* __restrict__ Sp, WfState W,
                                                                          QEnt* const* __restrict__ queues, uint32_t it,
                                                                          double* __restrict__ rad, DCamera C, PathParams P,
                                                                          InjParams I) {
    DScene Sv;
    if constexpr (LOBJ) lds_scene(Sp, Sv, false);  // filled in the first pass of the loop below
    const DScene& S = LOBJ ? Sv : *Sp;  // otherwise the scene in device memory (no by-value copy in scratch)
    __shared__ int stk_all[stack_lds(SM) * kBlock];
    const StkT<OVF, stack_lds(SM)> stk = make_stk<OVF, stack_lds(SM)>(S, stk_all);
    // the spheres mode reads its tree top from LDS (s_top4)
    constexpr bool kTop = SM == kSmSpheres && kLTop > 0;
    uint32_t* cnt = W.counts + (size_t)it * kWfsStride;
    const uint32_t nf = cnt[cix(kCntFront)];
    const uint32_t n_old = PART == kExtCamera ? 0u : nf + cnt[cix(kCntBack)];
    const uint32_t n = n_old + (PART == kExtCarried ? 0u : I.n_new);
    if (PART != kExtCamera && blockIdx.x == 0 && threadIdx.x == 0) cnt[0] = n_old;  // paths carried in (stats)
    const WfSet& cur = W.set[it & 1];
    const uint32_t base0 = blockIdx.x * kBlock;
    for (uint32_t base = base0; base < n; base += gridDim.x * kBlock) {
        // thread -> record: the front run [0, nf), the back run from the set's end down, then the
        // injected camera samples, whose records follow the front run
        const uint32_t j = base + threadIdx.x;
        const bool gen = PART == kExtCamera || (PART == kExtAll && j >= n_old);
        const uint32_t i = gen ? nf + (j - n_old) : j < nf ? j : W.cap - 1u - (j - nf);
        int cls = -1, qbp = 0;
        double qt = 0.0;  // the queue entry's hit (cls >= 0)
        bool live = false;
        Ray r;
        Rng rng;
        uint32_t item = 0;
        if (j < n) {
            if (gen) {
                uint64_t g, key;
                inj_sample(I, P, j - n_old, g, key, item);
                live = camera_sample(C, P, key, g, r, rng);
                if (!live) put_rad(rad, item, 0.0, 0.0, 0.0);
            } else {
                r = load_ray(cur, i, W.tagw);
                live = true;
            }
        }
        // the LDS image is filled once the block's first records are requested: their latency and the
        // image's overlap at the barrier (the spheres mode's tree top likewise)
        if constexpr (LOBJ)
            if (base == base0) lds_fill(S);
        if constexpr (kTop)
            if (base == base0) {
                const uint32_t nq = (uint32_t)S.ltop * (sizeof(DNode4) / 16);
                const uint4* __restrict__ src = (const uint4*)S.nodes4;
                for (uint32_t q = threadIdx.x; q < nq; q += kBlock) ((uint4*)s_top4)[q] = src[q];
                __syncthreads();
            }
        if (live) {
            double bend = RS_INF;
            // the spheres mode keeps the winner's t (the queue entry: the shading's sphere_rec_at), the others the range end
            constexpr bool kT = SM == kSmSpheres;
            const int bp = traverse<SM, StkT<OVF, stack_lds(SM)>, LOBJ, kT, kTop>(S, r, 0.0001, bend, stk);
            V3 add;
            bool done = true;
            if (bp < 0) {  // sky miss: L + T * background (camera.rs:253-254)
                add = background(S, r);
            } else {
                cls = (int)S.pclass[bp];
                if (cls == kClsLight) {  // DiffuseLight: emitted, scatter None (camera.rs:172-176,250)
                    Hit h;
                    int mi;
                    if (SM == kSmSpheres) {
                        const DPrim Pr = S.prims[bp];
                        sphere_rec_at(S.spheres[Pr.idx], Pr.mat, r, bend, h);  // bend: the winner's t (kT)
                        mi = Pr.mat;
                    } else {
                        // emission reads the record's material and point only: for a leaf object
                        // (a light class is only given to leaf objects and TfFacades of them) from
                        // its t-only test, without inlining the nested-object code a second time
                        if (S.prims[bp].kind != PK_XFORM) {
                            HitT ht;
                            Obj<0, 0>::hit_t(S, bp, r, 0.0001, bend, ht);
                            h.p = ht.p;
                            mi = S.prims[bp].mat;
                        } else {  // a TfFacade chain over a leaf (light-class prims are leafish)
                            finish_hit<SM, true>(S, bp, r, 0.0001, bend, h);
                            mi = h.mat;
                        }
                    }
                    add = emission<0>(S, S.mats[mi >= 0 ? mi : S.default_mat], h);
                    cls = -1;
                } else {
                    // a camera sample that goes on to shading: its record (T = 1, level 0), written from the
                    // registers it was traced from; a carried path's is in place. (Regenerating it in the
                    // shading instead measured 0.5 % slower on the bench frame and 5 % on C4: profiles/r5/ab.)
                    qbp = bp;
                    qt = bend;
                    if (gen) store_path(cur, i, r, v3(1.0, 1.0, 1.0), rng, item, 0u, W.tagw);
                    done = false;
                }
            }
            if (done) {  // 0 + T * add: the path's radiance so far is 0 (WfSet)
                D4 t4;
                if (gen) {
                    t4.x = t4.y = t4.z = 1.0;
                } else {
                    t4 = cur.thr[i];
                    item = W.tagw ? (uint32_t)(uint64_t)__double_as_longlong(cur.ray_o[i].w) : cur.tag[i].x;
                }
                put_rad(rad, item, 0.0 + t4.x * add.x, 0.0 + t4.y * add.y, 0.0 + t4.z * add.z);
            }
        }
#ifdef RS_TRAV_STATS
        {   // the wave's category: its first live lane's
            const int c = gen ? 0 : j < nf ? 1 : 2;
            const unsigned long long lm = __ballot(live);
            trav_stats_flush(live, lm ? __shfl(c, __ffsll((long long)lm) - 1, 64) : 0);
        }
#endif
        // the iteration's live camera samples are counted in the same block reduction (the carried
        // paths are cnt[0]), on one of kStatLines counters by block (one atomic per block on a single
        // word capped an empty camera-ray launch at ~88 atomics/us: 1.14 ms for 25.6 M samples, 0.10 ms
        // spread); launches without camera samples count nothing
        uint32_t* const cs[kClasses] = {&cnt[cix(1)], &cnt[cix(2)], &cnt[cix(3)], &cnt[cix(4)], &cnt[cix(5)]};
        const uint32_t slot = block_slot<kClasses>(cls, cs, gen && live,
                                                   PART == kExtCarried ? nullptr : &cnt[cix(kCntStat0 + (int)(blockIdx.x % kStatLines))]);
        if (cls >= 0) {
            QEnt q;
            q.i = i; q.bp = qbp; q.t = qt;
            queues[cls][slot] = q;
        }
    }
}

// The streaming frame's finish (its last iteration, rs_host.cpp FrameSched: after the last injection and
// kFinishAfter wavefront iterations): every path still carried (set it&1, front and back runs) is traced to its
// end by one thread -- ray_color's remaining levels as the megakernel's trace_path runs them (world_hit +
// shade_step; a live path's radiance so far is 0, so the result is the same 0 + T * term as the wavefront's) --
// in one launch instead of depth - kFinishAfter small iterations whose launch gaps and per-launch latency the
// few surviving paths of a depth-50 frame would pay. Segments beyond each path's first go to the iteration's
// statistics lines (its first is counted as carried, cnt[0]).
// (bounded to 2 waves: unbounded, the nest-2 instance took 256 VGPRs + 10 AGPRs at one wave per SIMD)
template <int SM, bool LOBJ>
__global__ __launch_bounds__(kBlock, 2) void k_wfs_finish(const DScene* __restrict__ Sp, WfState W, uint32_t it, uint32_t depth,
                                                      double* __restrict__ rad) {
    DScene Sv;
    if constexpr (LOBJ) lds_scene(Sp, Sv);
    const DScene& S = LOBJ ? Sv : *Sp;
    __shared__ int stk_all[stack_lds(SM) * kBlock];
    const StkT<true, stack_lds(SM)> stk = make_stk<true, stack_lds(SM)>(S, stk_all);
    uint32_t* cnt = W.counts + (size_t)it * kWfsStride;
    const uint32_t nf = cnt[cix(kCntFront)];
    const uint32_t n = nf + cnt[cix(kCntBack)];
    if (blockIdx.x == 0 && threadIdx.x == 0) cnt[0] = n;  // paths carried in (stats)
    const WfSet& cur = W.set[it & 1];
    uint32_t extra = 0;
    for (uint32_t base = blockIdx.x * kBlock; base < n; base += gridDim.x * kBlock) {
        const uint32_t j = base + threadIdx.x;
        if (j >= n) continue;
        const uint32_t i = j < nf ? j : W.cap - 1u - (j - nf);
        Ray r;
        V3 T;
        Rng rng;
        uint2 tg;
        load_path(cur, i, r, T, rng, W.tagw, tg);
        V3 L = v3(0.0, 0.0, 0.0);
        bool open = true;
        for (uint32_t lvl = tg.y; lvl < depth; ++lvl) {
            if (lvl != tg.y) ++extra;
            Hit h;
            double bend;
            const int bp = traverse<SM, StkT<true, stack_lds(SM)>, LOBJ>(S, r, 0.0001, bend, stk);  // world_hit
            const bool ok = finish_hit<SM>(S, bp, r, 0.0001, bend, h);
            if (!shade_step<SM>(S, ok, h, r, T, L, rng)) { open = false; break; }
        }
        if (open) L = close_path(L, T);  // depth limit: the next level would return 0
        put_rad(rad, tg.x, L.x, L.y, L.z);
    }
    // the extra segments, one atomic per wave on the iteration's statistics lines
    unsigned long long e = extra;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) e += __shfl_xor(e, off, 64);
    if ((threadIdx.x & 63) == 0 && e) atomicAdd(&cnt[cix(kCntStat0 + (int)(blockIdx.x % kStatLines))], (uint32_t)e);
}

// One batch of 256 queued paths of material class KIND (-1: the generic material switch; entries
// base .. base + 255 of a queue of n): finish the hit record, scatter, write the radiance of paths that
// end and append the survivors to the next set. Must be called by every thread of the block (block_slot).
template <int KIND, int SM>
__device__ __forceinline__ void wfs_shade_batch(const DScene& S, const WfState& W, const QEnt* __restrict__ queue,
                                                uint32_t n, uint32_t base, uint32_t it, uint32_t* cnt_next, uint32_t depth,
                                                double* __restrict__ rad) {
    const WfSet& cur = W.set[it & 1];
    const WfSet& nxt = W.set[(it + 1) & 1];
    const uint32_t j = base + threadIdx.x;
    bool alive = false;
    int light_ray = 0;
    Ray r;
    V3 T;
    Rng rng;
    uint32_t item = 0, lvl = 0;
    if (j < n) {
        const QEnt q = queue[j];
        const uint32_t i = q.i;
        uint2 tg;
        load_path(cur, i, r, T, rng, W.tagw, tg);
        item = tg.x;
        lvl = tg.y;
        const int bp = q.bp;
        Hit h;
        if constexpr (SM == kSmSpheres) {  // q.t: the winner's t (k_wfs_extend kT)
            const DPrim P = S.prims[bp];
            sphere_rec_at(S.spheres[P.idx], P.mat, r, q.t, h);
        } else {
            finish_hit<SM, (KIND >= 0)>(S, bp, r, 0.0001, q.t, h);
        }
        const int mi = h.mat >= 0 ? h.mat : S.default_mat;
        const DMaterial& M0 = S.mats[mi];
        bool cont;
        if (KIND >= 0) {
            cont = shade_surface<KIND, SM>(S, h, M0, M0, r, T, rng, &light_ray);
        } else if (M0.kind == RS_MAT_DIFFUSE_LIGHT) {
            // a composite prim whose record carries a light material (class 4): emitted, scatter
            // None (camera.rs:172-176, 250), 0 + T * e as in shade_step
            const V3 e = emission<0>(S, M0, h);
            const V3 L = v3(0.0, 0.0, 0.0) + v3(T.x * e.x, T.y * e.y, T.z * e.z);
            put_rad(rad, item, L.x, L.y, L.z);
            cont = false;
            item = ~0u;  // radiance written
        } else {
            int ms = mi;
            for (int k = 0; k < 16 && S.mats[ms].kind == RS_MAT_MIXED; ++k) {  // mixed_material.rs:43-50
                const DMaterial& X = S.mats[ms];
                ms = ((double)rng.next_u32() < 4294967295.0 * X.mix_p) ? X.mix_a : X.mix_b;
            }
            cont = shade_surface<-1, SM>(S, h, M0, S.mats[ms], r, T, rng, &light_ray);
        }
        alive = cont && (lvl + 1 < depth);  // the depth limit of ray_color (camera.rs:161)
        if (!alive && item != ~0u) {  // absorbed or depth limit: no emission term
            const V3 L = close_path(v3(0.0, 0.0, 0.0), T);
            put_rad(rad, item, L.x, L.y, L.z);
        }
    }
    // light-sample rays (camera.rs:196-205, all aimed at the few lights) fill the next set from
    // the front, the rest from the back: the next extend's waves then trace rays of one kind
    // (the other rays binned by direction sign inside each block's back-run slots, 2 / 4 / 8 bins: bench frame -0.6 /
    // 0.0 / +0.4 %, the N = 8 share and C2 / C3 shapes unchanged: profiles/r6/ab/bsdf_bins_r7d.txt, not kept)
    uint32_t* const gc[2] = {&cnt_next[cix(kCntBack)], &cnt_next[cix(kCntFront)]};
    const uint32_t slot = block_slot<2>(alive ? light_ray : -1, gc);
    if (alive) {
        const uint32_t p = light_ray ? slot : W.cap - 1u - slot;
        store_path(nxt, p, r, T, rng, item, lvl + 1u, W.tagw);
    }
}

// Every material class of an iteration in ONE launch: the grid walks the concatenation of the class
// queues' 256-path batches (class 0's, then class 1's, ...); a block's class is uniform, so each batch
// runs its class's specialised code. One launch per iteration instead of one per class removes the
// per-class launch tails (the small classes' queues take 5-50 us each however short they are).
// G4: the scene has class-4 prims (the generic material switch, composite objects), compiled in only
// then (it sets the kernel's register count). LOBJ: the scene's tables from its LDS image (lds_scene).
// Waves: 3; nest-2 with class 4 and the tables in global memory 1 (bounded to 3 it spilled and lost
// 21 % on C4 in round 3; with the LDS image 3 waves measured 5 % faster than 2: nest2_registers; the heavy
// launch alone at 2 waves: C4 5.43 -> 5.38 Gseg/s, profiles/r5/ab/c4_waves_r5l)
// PS: the classes of this launch -- 0 all; 1 the lean ones (Lambertian, Metal, Dielectric: bounded to 4 waves);
// 2 the heavy ones (DiffuseMetal's two ONBs and ReflectionPdf loop, the generic switch): rs_scene::shade_split
template <int SM, bool G4, bool LOBJ, int PS>
// (the nest-2 lean launch at 3 waves, no scratch: C4-shaped frame +0.4 %; at 5 waves +5.7 %:
// profiles/r5/ab/n2_lean_waves_r6d.jsonl)
// (the spheres lean launch at 5 waves spills 136 B: bench frame +10 %, profiles/r6/ab/waves_cam_lean_r7i.txt)
#define RS_SHADE_WAVES(SM, G4, LOBJ, PS) (PS == 1 ? 4 : (SM == kSmNest2 && G4 && !LOBJ) ? 1 : 3)
__global__ __launch_bounds__(kBlock, RS_SHADE_WAVES(SM, G4, LOBJ, PS)) void k_wfs_shade_all(const DScene* __restrict__ Sp, WfState W,
                                                                                   QEnt* const* __restrict__ queues,
                                                                                   uint32_t class_mask, uint32_t it,
                                                                                   uint32_t depth,
                                                                                   double* __restrict__ rad) {
    // (3 waves: 171 -> 168 VGPRs; at 4 waves it spilled 156 B, +6 %; nest-2 bounded at 3 spilled: C4 -21 %)
    DScene Sv;
    if constexpr (LOBJ) lds_scene(Sp, Sv);
    const DScene& S = LOBJ ? Sv : *Sp;
    const uint32_t* cnt = W.counts + (size_t)it * kWfsStride;
    uint32_t* cnt_next = W.counts + (size_t)(it + 1) * kWfsStride;
    constexpr int NC = G4 ? 5 : 4;
    constexpr uint32_t kPart = PS == 0 ? 0x1fu : PS == 1 ? 0x0bu : 0x14u;  // classes of this launch
    uint32_t n[NC], first[NC + 1];
    first[0] = 0;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
        n[k] = ((class_mask & kPart) >> k & 1u) ? cnt[cix(1 + k)] : 0u;
        first[k + 1] = first[k] + (n[k] + kBlock - 1) / kBlock;
    }
    for (uint32_t v = blockIdx.x; v < first[NC]; v += gridDim.x) {
        int k = 0;
#pragma unroll
        for (int c = 1; c < NC; ++c) k += v >= first[c] ? 1 : 0;
        const uint32_t base = (v - first[k]) * kBlock;
        if (k == 0) {
            if constexpr ((kPart & 1u) != 0)
                wfs_shade_batch<RS_MAT_LAMBERTIAN, SM>(S, W, queues[0], n[0], base, it, cnt_next, depth, rad);
        } else if (k == 1) {
            if constexpr ((kPart & 2u) != 0)
                wfs_shade_batch<RS_MAT_METAL, SM>(S, W, queues[1], n[1], base, it, cnt_next, depth, rad);
        } else if (k == 2) {
            if constexpr ((kPart & 4u) != 0)
                wfs_shade_batch<RS_MAT_DIFFUSE_METAL, SM>(S, W, queues[2], n[2], base, it, cnt_next, depth, rad);
        } else if (k == 3 || !G4) {
            if constexpr ((kPart & 8u) != 0)
                wfs_shade_batch<RS_MAT_DIELECTRIC, SM>(S, W, queues[3], n[3], base, it, cnt_next, depth, rad);
        } else {
            if constexpr ((kPart & 16u) != 0)
                wfs_shade_batch<-1, SM>(S, W, queues[NC - 1], n[NC - 1], base, it, cnt_next, depth, rad);
        }
    }
}


#if RS_TU_COMMON
// painter.rs:167-179: a pixel's sum over its samples, in sample order. One thread per (pixel,
// channel), the batch's samples read 16 at a time (the adds stay in order): a strong-scaled share of
// a frame has few pixels, and a thread per pixel looping over 3 x N dependent loads left the kernel
// latency-bound (80 us for the N = 8 share of the bench frame).
__global__ __launch_bounds__(kBlock) void k_accumulate(const double* __restrict__ rad, double* __restrict__ acc,
                                                      uint32_t n_pix, uint32_t n_samp, int first, int last, FinalParams P,
                                                      float* __restrict__ out, uint32_t* __restrict__ zero, uint32_t n_zero) {
    const uint64_t t = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    // the frame's queue counters, read by no kernel after this one: reset for the next frame
    // (rs_host.cpp counts_clean; the host passes n_zero = 0 when it still reads them)
    for (uint64_t z = t; z < n_zero; z += (uint64_t)gridDim.x * kBlock) zero[z] = 0u;
    if (t >= 3ull * n_pix) return;
    // thread 3p + c: a wave's reads of a sample plane of the item-major radiance are contiguous
    const uint32_t p = (uint32_t)(t / 3), c = (uint32_t)(t - 3ull * p);
    double a = first ? 0.0 : acc[(uint64_t)c * n_pix + p];
    const double* rc = rad + 3ull * p + c;
    const uint64_t sstep = 3ull * n_pix;
    uint32_t s = 0;
    for (; s + 16 <= n_samp; s += 16) {
        double v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = rc[(uint64_t)(s + k) * sstep];
#pragma unroll
        for (int k = 0; k < 16; ++k) a = a + v[k];
    }
    for (; s < n_samp; ++s) a = a + rc[(uint64_t)s * sstep];
    if (!last) {
        acc[(uint64_t)c * n_pix + p] = a;
        return;
    }
    // the last batch: into_color of this channel (k_finalize's arithmetic) straight into the frame
    const uint32_t x = p % P.width;
    const uint32_t y = P.row_begin + (p / P.width) * P.row_step;
    const uint64_t pix = (uint64_t)y * P.width + x;
    const bool masked = P.mask && !P.mask[pix];
    double v = a / (double)P.n_samples;
    if (P.gamma) v = sqrt(v);
    out[pix * 4 + c] = masked ? 0.0f : (float)v;
    if (c == 0) out[pix * 4 + 3] = masked ? 0.0f : 1.0f;
}
#endif  // RS_TU_COMMON

#if RS_TU_COMMON
__global__ __launch_bounds__(kBlock) void k_finalize(const double* __restrict__ acc, float* __restrict__ out, FinalParams P) {
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= P.n_pix_local) return;
    const uint32_t x = p % P.width;
    const uint32_t y = P.row_begin + (p / P.width) * P.row_step;
    const uint64_t pix = (uint64_t)y * P.width + x;
    float4 o;
    if (P.mask && !P.mask[pix]) {
        o = make_float4(0.f, 0.f, 0.f, 0.f);
    } else {
        const double n = (double)P.n_samples;
        double r = acc[p] / n, g = acc[(uint64_t)P.n_pix_local + p] / n, b = acc[2ull * P.n_pix_local + p] / n;
        if (P.gamma) { r = sqrt(r); g = sqrt(g); b = sqrt(b); }
        o = make_float4((float)r, (float)g, (float)b, 1.0f);
    }
    reinterpret_cast<float4*>(out)[pix] = o;
}
#endif  // RS_TU_COMMON

#if RS_TU_COMMON
// ---- progressive passes (src/bin/raysnail.rs:176-208, 150-173, 394-422) ----
__global__ __launch_bounds__(kBlock) void k_combine(float4* __restrict__ acc, const float4* __restrict__ nw, uint64_t n,
                                                   float p) {
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const float4 v = nw[i];
    if (v.x == 0.f && v.y == 0.f && v.z == 0.f && v.w == 0.f) return;  // no new data: keep old
    const float4 o = acc[i];
    const float d = p + 1.0f;
    acc[i] = make_float4((o.x * p + v.x) / d, (o.y * p + v.y) / d, (o.z * p + v.z) / d, (o.w * p + v.w) / d);
}
#endif  // RS_TU_COMMON

// one pixel's calc_noise: sum over the 5x5 window of color_diff(def, neighbour), window rows
// y-2..y+2 (outer) and columns y-2..y+2 (inner; upstream shadows x with y), outside = def
__device__ __forceinline__ float calc_noise(const float4* px, int x, int y, int w, int h) {
    const float4 def = px[(size_t)y * w + x];
    float diff = 0.0f;
    const int cx = y;
    for (int yy = y - 2; yy < y + 3; ++yy)
        for (int xx = cx - 2; xx < cx + 3; ++xx) {
            float4 q = def;
            if (xx >= 0 && yy >= 0 && xx < w && yy < h) q = px[(size_t)yy * w + xx];
            const float rd = def.x - q.x, gd = def.y - q.y, bd = def.z - q.z;
            diff += rd * rd + gd * gd + bd * bd;
        }
    return diff;
}

#if RS_TU_COMMON
__global__ __launch_bounds__(kBlock) void k_noise(const float4* __restrict__ px, int w, int h, float t,
                                                 uint8_t* __restrict__ redo, unsigned int* __restrict__ mm,
                                                 unsigned long long* __restrict__ count) {
    __shared__ unsigned int s_cnt;
    if (threadIdx.x == 0) s_cnt = 0;
    __syncthreads();
    const uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i < (uint64_t)w * h) {
        const int x = (int)(i % w), y = (int)(i / w);
        const float n = calc_noise(px, x, y, w, h);
        const bool r = n >= t;
        if (redo) redo[i] = r ? 1 : 0;
        if (r) atomicAdd(&s_cnt, 1u);
        // min / max over non-negative floats (or NaN, which the reference's `<` / `>` skip)
        if (n == n) {
            atomicMin(&mm[0], __float_as_uint(n));
            atomicMax(&mm[1], __float_as_uint(n));
        }
    }
    __syncthreads();
    if (threadIdx.x == 0 && s_cnt) atomicAdd(count, (unsigned long long)s_cnt);
}
#endif  // RS_TU_COMMON

#if RS_TU_COMMON
// Diagnostic: World::hit for a batch of rays (tests/ per-primitive parity probes).
// rays[i] = o(3) d(3) time; out[i] = hit t1 t2 p(3) n(3) 0 0 outside mat  (13 doubles, oracle layout)
__global__ __launch_bounds__(kBlock) void k_probe_hit(const DScene* __restrict__ Sp, const double* __restrict__ rays, uint32_t n, double tmin,
                                                     double tmax, double* __restrict__ out) {
    const DScene& S = *Sp;  // the scene lives in device memory: no by-value copy in scratch
    __shared__ int stk_all[kStackMax * kBlock];
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    Ray r;
    r.o = ld3(rays + 7 * i); r.d = ld3(rays + 7 * i + 3); r.time = rays[7 * i + 6];
    r.key = 0;  // probe rays: medium key 0 (orc_world_hit likewise)
    Hit h;
    double* o = out + 13 * (size_t)i;
    for (int k = 0; k < 13; ++k) o[k] = 0.0;
    // range end handled by clamping best: world_hit starts from +inf, so emulate [tmin, tmax) by a
    // post-check only when tmax is infinite (the render path always passes +inf)
    if (world_hit<kSmGeneric>(S, r, tmin, h, make_stk(S, stk_all)) && h.t1 < tmax) {
        o[0] = 1.0; o[1] = h.t1; o[2] = h.t2;
        o[3] = h.p.x; o[4] = h.p.y; o[5] = h.p.z; o[6] = h.n.x; o[7] = h.n.y; o[8] = h.n.z;
        if (S.uv) { o[9] = h.u; o[10] = h.v; }  // (u, v) exist only in scenes that read them
        o[11] = h.outside ? 1.0 : 0.0; o[12] = (double)h.mat;
    }
}
#endif  // RS_TU_COMMON

// Diagnostic: the radiance and world.hit count of samples s0 .. s0+n-1 of pixel (x, y), each
// through the megakernel's trace_path (tests/ per-sample parity; the oracle's orc_sample_radiance).
template <int SM>
__global__ __launch_bounds__(kBlock) void k_probe_sample(const DScene* __restrict__ Sp, DCamera C, PathParams P, uint32_t x, uint32_t y,
                                                        uint32_t s0, uint32_t n, double* __restrict__ out) {
    const DScene& S = *Sp;  // the scene lives in device memory: no by-value copy in scratch
    __shared__ int stk_all[kStackMax * kBlock];
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    Ray r;
    Rng rng;
    camera_sample_xy(C, P, P.key_base, x, y, s0 + i, r, rng);
    uint32_t segs = 0;
    const V3 L = trace_path<SM>(S, r, P.depth, rng, make_stk(S, stk_all), segs);
    out[4 * (size_t)i] = L.x; out[4 * (size_t)i + 1] = L.y; out[4 * (size_t)i + 2] = L.z;
    out[4 * (size_t)i + 3] = (double)segs;
}

// ---- launchers ----
// Mode-dependent launchers: launch_X_sm<SM> (defined and instantiated per mode unit) behind a
// dispatcher on the scene mode (common unit).
#define RS_SM_LAUNCHERS(X)                                                                                     \
    X(hipError_t, probe_sample, (const SceneRef& s, const DCamera& c, const PathParams& p, uint32_t x, uint32_t y,  \
                                 uint32_t s0, uint32_t n, double* out, hipStream_t st), (s, c, p, x, y, s0, n, out, st)) \
    X(hipError_t, path_mega, (const SceneRef& s, const DCamera& c, const PathParams& p, double* rad,              \
                              unsigned long long* seg_counters, uint32_t max_blocks, hipStream_t st),             \
      (s, c, p, rad, seg_counters, max_blocks, st))                                                            \
    X(hipError_t, wf_extend, (const SceneRef& s, const WfState& w, uint32_t bounce, uint32_t blocks, hipStream_t st), \
      (s, w, bounce, blocks, st))                                                                              \
    X(hipError_t, wf_shade, (const SceneRef& s, const WfState& w, uint32_t bounce, uint32_t depth, uint64_t n_items,  \
                             double* rad, uint32_t blocks, hipStream_t st), (s, w, bounce, depth, n_items, rad, blocks, st)) \
    X(hipError_t, wf_occupancy, (int* e, int* sh), (e, sh))
#define RS_SORTED_LAUNCHERS(X)                                                                                 \
    X(hipError_t, wfs_extend, (const SceneRef& s, const DCamera& c, const PathParams& p, const WfState& w,       \
                               QEnt* const* queues, uint32_t it, const InjParams& inj, double* rad, uint32_t blocks, \
                               int part, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1),                        \
      (s, c, p, w, queues, it, inj, rad, blocks, part, st, ev0, ev1))                                                  \
    X(hipError_t, wfs_finish, (const SceneRef& s, const WfState& w, uint32_t it, uint32_t depth, double* rad,        \
                               uint32_t blocks, hipStream_t st), (s, w, it, depth, rad, blocks, st))              \
    X(hipError_t, wfs_shade_all, (const SceneRef& s, const WfState& w, QEnt* const* queues, uint32_t class_mask, \
                                  uint32_t it, uint32_t depth, double* rad, uint32_t blocks, bool split, \
                                  hipStream_t st),                                                              \
      (s, w, queues, class_mask, it, depth, rad, blocks, split, st))
#define RS_DECLARE_SM(R, NAME, PARAMS, ARGS) template <int SMC> R NAME##_sm PARAMS;
RS_SM_LAUNCHERS(RS_DECLARE_SM)
RS_SORTED_LAUNCHERS(RS_DECLARE_SM)

#if RS_TU_MODES
template <int SMC>
hipError_t probe_sample_sm(const SceneRef& s, const DCamera& c, const PathParams& p, uint32_t x, uint32_t y, uint32_t s0,
                           uint32_t n, double* out, hipStream_t st) {
    const uint32_t blocks = (n + kBlock - 1) / kBlock;
    if (!blocks) return hipSuccess;
    hipLaunchKernelGGL(k_probe_sample<SMC>, dim3(blocks), dim3(kBlock), 0, st, s.dev, c, p, x, y, s0, n, out);
    return hipGetLastError();
}

template <int SMC>
hipError_t path_mega_sm(const SceneRef& s, const DCamera& c, const PathParams& p, double* rad,
                        unsigned long long* seg_counters, uint32_t max_blocks, hipStream_t st) {
    const uint64_t blocks = std::min<uint64_t>((p.n_items + kBlock - 1) / kBlock, max_blocks);
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_path_mega<SMC>, dim3((uint32_t)blocks), dim3(kBlock), 0, st, s.dev, c, p, rad, seg_counters);
    return hipGetLastError();
}

template <int SMC>
hipError_t wf_extend_sm(const SceneRef& s, const WfState& w, uint32_t bounce, uint32_t blocks, hipStream_t st) {
    if constexpr (SMC == kSmFlat) {
        if (flat_dyn(s)) {
            hipLaunchKernelGGL(k_wf_extend_dyn<SMC>, dim3(blocks), dim3(kBlock), 0, st, s.dev, w, bounce);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL(k_wf_extend<SMC>, dim3(blocks), dim3(kBlock), 0, st, s.dev, w, bounce);
    return hipGetLastError();
}

template <int SMC>
hipError_t wf_shade_sm(const SceneRef& s, const WfState& w, uint32_t bounce, uint32_t depth, uint64_t n_items,
                       double* rad, uint32_t blocks, hipStream_t st) {
    if constexpr (SMC == kSmFlat) {
        if (flat_lamb(s)) {
            hipLaunchKernelGGL((k_wf_shade<SMC, true>), dim3(blocks), dim3(kBlock), 0, st, s.dev, w, bounce, depth, n_items, rad);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL(k_wf_shade<SMC>, dim3(blocks), dim3(kBlock), 0, st, s.dev, w, bounce, depth, n_items, rad);
    return hipGetLastError();
}

template <int SMC>
hipError_t wf_occupancy_sm(int* e, int* sh) {
    const void* ext = reinterpret_cast<const void*>(&k_wf_extend<SMC>);
    if constexpr (SMC == kSmFlat) ext = reinterpret_cast<const void*>(&k_wf_extend_dyn<SMC>);
    hipError_t r = hipOccupancyMaxActiveBlocksPerMultiprocessor(e, ext, kBlock, 0);
    if (r == hipSuccess)
        r = hipOccupancyMaxActiveBlocksPerMultiprocessor(sh, reinterpret_cast<const void*>(&k_wf_shade<SMC>), kBlock, 0);
    return r;
}

// the LDS-only traversal stack (StkT<false>) where the tree allows it; spheres mode only (the other
// modes keep one instantiation each: compile time)
[[maybe_unused]] static inline bool lds_only_stack(const SceneRef& s, int sm) { return s.host->stack_need + 3 <= stack_lds(sm); }

template <int SMC>
hipError_t wfs_extend_sm(const SceneRef& s, const DCamera& c, const PathParams& p, const WfState& w, QEnt* const* queues,
                         uint32_t it, const InjParams& inj, double* rad, uint32_t blocks, int part, hipStream_t st,
                         hipEvent_t ev0, hipEvent_t ev1) {
    if (!blocks) return hipSuccess;
#define RS_EXT_LAUNCH(OVF, PART) RS_EXT_LAUNCH_L(OVF, PART, false, 0)
#define RS_EXT_LAUNCH_L(OVF, PART, LOBJ, SHM)                                                                        \
    hipExtLaunchKernelGGL((k_wfs_extend<SMC, OVF, PART, LOBJ>), dim3(blocks), dim3(kBlock), SHM, st, ev0, ev1, 0, s.dev, \
                          w, queues, it, rad, c, p, inj)
    // nest modes: the LDS image when the scene has one (the spheres mode has none: its 41 KB tree and
    // sphere records per block halved the extend's occupancy, bench frame 7.63 -> 9.94 ms)
    const uint32_t shm = s.host->limg_bytes;
    if constexpr (SMC == kSmNest2) {  // split launches only (ext_split)
        if (part == kExtCamera) { if (shm) RS_EXT_LAUNCH_L(true, kExtCamera, true, shm); else RS_EXT_LAUNCH(true, kExtCamera); }
        else { if (shm) RS_EXT_LAUNCH_L(true, kExtCarried, true, shm); else RS_EXT_LAUNCH(true, kExtCarried); }
    } else if constexpr (SMC == kSmNest0) {
        if (part == kExtAll) { if (shm) RS_EXT_LAUNCH_L(true, kExtAll, true, shm); else RS_EXT_LAUNCH(true, kExtAll); }
        else if (part == kExtCamera) { if (shm) RS_EXT_LAUNCH_L(true, kExtCamera, true, shm); else RS_EXT_LAUNCH(true, kExtCamera); }
        else { if (shm) RS_EXT_LAUNCH_L(true, kExtCarried, true, shm); else RS_EXT_LAUNCH(true, kExtCarried); }
    } else if constexpr (SMC == kSmSpheres) {
        const bool lds = lds_only_stack(s, SMC);
        if (part == kExtAll) { if (lds) RS_EXT_LAUNCH(false, kExtAll); else RS_EXT_LAUNCH(true, kExtAll); }
        else if (part == kExtCamera) { if (lds) RS_EXT_LAUNCH(false, kExtCamera); else RS_EXT_LAUNCH(true, kExtCamera); }
        else { if (lds) RS_EXT_LAUNCH(false, kExtCarried); else RS_EXT_LAUNCH(true, kExtCarried); }
    } else {
        if (part == kExtAll) RS_EXT_LAUNCH(true, kExtAll);
        else if (part == kExtCamera) RS_EXT_LAUNCH(true, kExtCamera);
        else RS_EXT_LAUNCH(true, kExtCarried);
    }
#undef RS_EXT_LAUNCH
#undef RS_EXT_LAUNCH_L
    return hipGetLastError();
}

template <int SMC>
hipError_t wfs_finish_sm(const SceneRef& s, const WfState& w, uint32_t it, uint32_t depth, double* rad, uint32_t blocks,
                         hipStream_t st) {
    if (!blocks) return hipSuccess;
    const uint32_t shm = s.host->limg_bytes;  // nest modes' LDS image
    if constexpr (SMC == kSmNest0 || SMC == kSmNest2) {
        if (shm) {
            hipLaunchKernelGGL((k_wfs_finish<SMC, true>), dim3(blocks), dim3(kBlock), shm, st, s.dev, w, it, depth, rad);
            return hipGetLastError();
        }
    }
    hipLaunchKernelGGL((k_wfs_finish<SMC, false>), dim3(blocks), dim3(kBlock), 0, st, s.dev, w, it, depth, rad);
    return hipGetLastError();
}

template <int SMC>
hipError_t wfs_shade_all_sm(const SceneRef& s, const WfState& w, QEnt* const* queues, uint32_t class_mask, uint32_t it,
                            uint32_t depth, double* rad, uint32_t blocks, bool split, hipStream_t st) {
    if (!blocks) return hipSuccess;
#define RS_SHADE_LAUNCH(G4, LOBJ, PS, SHM)                                                                          \
    hipLaunchKernelGGL((k_wfs_shade_all<SMC, G4, LOBJ, PS>), dim3(blocks), dim3(kBlock), SHM, st, s.dev, w, queues, \
                       class_mask, it, depth, rad)
    const uint32_t shm = s.host->limg_bytes;  // nest modes' LDS image (none in the spheres mode)
    if constexpr (SMC == kSmNest0 || SMC == kSmNest2) {
        // with the LDS image: the lean classes (leaf objects, classes 0-3 but DiffuseMetal) at 4 waves (128 VGPRs, 44 B
        // of scratch), then DiffuseMetal and the composites (class 4: the nested-object record) at 3 (C4-shaped frame
        // 113.2 -> 111.8 ms, profiles/r5/ab/c4_split_r5h.jsonl)
        if (split && shm) {
            RS_SHADE_LAUNCH(false, true, 1, shm);
            if (class_mask & 0x14u) {
                if (class_mask & (1u << 4)) RS_SHADE_LAUNCH(true, true, 2, shm);
                else RS_SHADE_LAUNCH(false, true, 2, shm);
            }
            return hipGetLastError();
        }
        if (class_mask & (1u << 4)) { if (shm) RS_SHADE_LAUNCH(true, true, 0, shm); else RS_SHADE_LAUNCH(true, false, 0, 0); }
        else { if (shm) RS_SHADE_LAUNCH(false, true, 0, shm); else RS_SHADE_LAUNCH(false, false, 0, 0); }
    } else if (split) {
        // the lean classes (Lambertian, Metal, Dielectric) at 4 waves, then the heavy ones (DiffuseMetal, the
        // generic switch) at 3: the merged kernel's registers are DiffuseMetal's (168), Lambertian's alone 133
        RS_SHADE_LAUNCH(false, false, 1, 0);
        if (class_mask & 0x14u) {
            if (class_mask & (1u << 4)) RS_SHADE_LAUNCH(true, false, 2, 0);
            else RS_SHADE_LAUNCH(false, false, 2, 0);
        }
    } else {
        if (class_mask & (1u << 4)) RS_SHADE_LAUNCH(true, false, 0, 0);
        else RS_SHADE_LAUNCH(false, false, 0, 0);
    }
#undef RS_SHADE_LAUNCH
    return hipGetLastError();
}
#endif  // RS_TU_MODES

#if defined(RS_TU) && RS_TU >= 0  // this unit's mode
#define RS_INSTANTIATE_SM(R, NAME, PARAMS, ARGS) template R NAME##_sm<RS_TU> PARAMS;
RS_SM_LAUNCHERS(RS_INSTANTIATE_SM)
#if RS_TU == 1 || RS_TU == 3 || RS_TU == 4  // the streaming-wavefront modes
RS_SORTED_LAUNCHERS(RS_INSTANTIATE_SM)
#endif
#endif

#if RS_TU_COMMON
#define RS_DISPATCH_ALL(R, NAME, PARAMS, ARGS) \
    R launch_##NAME PARAMS_SM_##NAME { RS_SM_DISPATCH(sm, return NAME##_sm<SMC> ARGS); return hipErrorInvalidValue; }
hipError_t launch_probe_sample(const SceneRef& s, const DCamera& c, const PathParams& p, int sm, uint32_t x, uint32_t y,
                               uint32_t s0, uint32_t n, double* out, hipStream_t st) {
    RS_SM_DISPATCH(sm, return probe_sample_sm<SMC>(s, c, p, x, y, s0, n, out, st));
    return hipErrorInvalidValue;
}

hipError_t launch_path_mega(const SceneRef& s, const DCamera& c, const PathParams& p, int sm, double* rad,
                            unsigned long long* seg_counters, uint32_t max_blocks, hipStream_t st) {
    RS_SM_DISPATCH(sm, return path_mega_sm<SMC>(s, c, p, rad, seg_counters, max_blocks, st));
    return hipErrorInvalidValue;
}

hipError_t launch_wf_gen(const DCamera& c, const PathParams& p, const WfState& w, uint64_t item0, uint32_t n, double* rad,
                         hipStream_t st) {
    const uint32_t blocks = (n + kBlock - 1) / kBlock;
    if (!blocks) return hipSuccess;
    hipLaunchKernelGGL(k_wf_gen, dim3(blocks), dim3(kBlock), 0, st, c, p, w, item0, n, rad);
    return hipGetLastError();
}

hipError_t launch_wf_extend(const SceneRef& s, const WfState& w, uint32_t bounce, uint32_t blocks, int sm, hipStream_t st) {
    RS_SM_DISPATCH(sm, return wf_extend_sm<SMC>(s, w, bounce, blocks, st));
    return hipErrorInvalidValue;
}

hipError_t launch_wf_shade(const SceneRef& s, const WfState& w, uint32_t bounce, uint32_t depth, uint64_t n_items, double* rad,
                           uint32_t blocks, int sm, hipStream_t st) {
    RS_SM_DISPATCH(sm, return wf_shade_sm<SMC>(s, w, bounce, depth, n_items, rad, blocks, st));
    return hipErrorInvalidValue;
}

hipError_t wf_occupancy(int sm, int* e, int* sh) {
    RS_SM_DISPATCH(sm, return wf_occupancy_sm<SMC>(e, sh));
    return hipErrorInvalidValue;
}

hipError_t launch_wfs_extend(const SceneRef& s, const DCamera& c, const PathParams& p, const WfState& w,
                             QEnt* const* queues, uint32_t it, const InjParams& inj, double* rad, uint32_t blocks,
                             int part, int sm, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
    RS_SM_SORTED_DISPATCH(sm, return wfs_extend_sm<SMC>(s, c, p, w, queues, it, inj, rad, blocks, part, st, ev0, ev1));
    return hipErrorInvalidValue;
}

hipError_t launch_wfs_finish(const SceneRef& s, const WfState& w, uint32_t it, uint32_t depth, double* rad, uint32_t blocks,
                             int sm, hipStream_t st) {
    RS_SM_SORTED_DISPATCH(sm, return wfs_finish_sm<SMC>(s, w, it, depth, rad, blocks, st));
    return hipErrorInvalidValue;
}

hipError_t launch_wfs_shade_all(const SceneRef& s, const WfState& w, QEnt* const* queues, uint32_t class_mask,
                                uint32_t it, uint32_t depth, double* rad, uint32_t blocks, bool split, int sm,
                                hipStream_t st) {
    RS_SM_SORTED_DISPATCH(sm, return wfs_shade_all_sm<SMC>(s, w, queues, class_mask, it, depth, rad, blocks, split, st));
    return hipErrorInvalidValue;
}

hipError_t launch_combine(float* acc, const float* nw, uint64_t n, float p, hipStream_t st) {
    const uint64_t blocks = (n + kBlock - 1) / kBlock;
    if (!blocks) return hipSuccess;
    hipLaunchKernelGGL(k_combine, dim3((uint32_t)blocks), dim3(kBlock), 0, st, reinterpret_cast<float4*>(acc),
                       reinterpret_cast<const float4*>(nw), n, p);
    return hipGetLastError();
}

hipError_t launch_noise(const float* px, int w, int h, float t, uint8_t* redo, unsigned int* mm,
                        unsigned long long* count, hipStream_t st) {
    const uint64_t n = (uint64_t)w * h;
    const uint64_t blocks = (n + kBlock - 1) / kBlock;
    if (!blocks) return hipSuccess;
    hipLaunchKernelGGL(k_noise, dim3((uint32_t)blocks), dim3(kBlock), 0, st, reinterpret_cast<const float4*>(px), w, h,
                       t, redo, mm, count);
    return hipGetLastError();
}

hipError_t launch_probe_hit(const SceneRef& s, const double* rays, uint32_t n, double tmin, double tmax, double* out,
                            hipStream_t st) {
    const uint32_t blocks = (n + kBlock - 1) / kBlock;
    if (!blocks) return hipSuccess;
    hipLaunchKernelGGL(k_probe_hit, dim3(blocks), dim3(kBlock), 0, st, s.dev, rays, n, tmin, tmax, out);
    return hipGetLastError();
}

hipError_t launch_accumulate(const double* rad, double* acc, uint32_t n_pix, uint32_t n_samp_batch,
                             int first_batch, int last_batch, const FinalParams& p, float* out_rgba, uint32_t* zero,
                             uint32_t n_zero, hipStream_t st) {
    const uint32_t blocks = (uint32_t)((3ull * n_pix + kBlock - 1) / kBlock);
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_accumulate, dim3(blocks), dim3(kBlock), 0, st, rad, acc, n_pix, n_samp_batch, first_batch,
                       last_batch, p, out_rgba, zero, n_zero);
    return hipGetLastError();
}

hipError_t launch_finalize(const double* acc, float* out_rgba, const FinalParams& p, hipStream_t st) {
    const uint32_t blocks = (p.n_pix_local + kBlock - 1) / kBlock;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_finalize, dim3(blocks), dim3(kBlock), 0, st, acc, out_rgba, p);
    return hipGetLastError();
}
#endif  // RS_TU_COMMON

}  // namespace rs

#if defined(RS_TRAV_STATS)
#if !defined(RS_TU)
#define RS_TS_FN rs_debug_trav_stats
#elif RS_TU < 0
#define RS_TS_FN rs_debug_trav_stats_c
#elif RS_TU == 0
#define RS_TS_FN rs_debug_trav_stats_0
#elif RS_TU == 1
#define RS_TS_FN rs_debug_trav_stats_1
#elif RS_TU == 2
#define RS_TS_FN rs_debug_trav_stats_2
#elif RS_TU == 3
#define RS_TS_FN rs_debug_trav_stats_3
#else
#define RS_TS_FN rs_debug_trav_stats_4
#endif
extern "C" int RS_TS_FN(unsigned long long out[128], int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(rs::g_trav_stats), 128 * sizeof(unsigned long long)) != hipSuccess) return -3;
    if (reset) {
        unsigned long long z[128] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(rs::g_trav_stats), z, sizeof(z)) != hipSuccess) return -3;
    }
    return 0;
}
#endif
