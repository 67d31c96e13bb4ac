// rs_kernels.hip — gfx950 kernels of the render path.
//
//   k_path_mega   painter.rs:154-187 (render_pixel, one sample) -> camera.rs:77-85 (Camera::ray)
//                 -> camera.rs:156-255 (ray_color, iterated) with BVH traversal (bvh.rs:173-192)
//   k_accumulate  painter.rs:167-179 color_vec sum, in sample order
//   k_finalize    vec3.rs:227-240 into_color (/N, sqrt gamma, f32, alpha 1) + painter.rs:204-210 mask
//
// Build with -ffp-contract=off (see Makefile): the f64 arithmetic mirrors the reference's
// operation order, so the only differences from the CPU oracle are ocml vs glibc ulps in
// sin/cos/pow (documented tolerance in DESIGN.md).
#include "rs_device.h"
#include "rs_internal.h"

namespace rs {

// aabb.rs:20-38 with inv = 1/d[i] precomputed per ray (the reference recomputes the same value
// per node). Branch-free form: max/min over the three axes is equivalent to the early-exit loop
// because t_min only grows and t_max only shrinks. Returns the entry distance in `entry`.
__device__ __forceinline__ bool slab(const double lo[3], const double hi[3], const V3& o, const V3& inv, double tmin,
                                     double tmax, double& entry) {
    double t0x = (lo[0] - o.x) * inv.x, t1x = (hi[0] - o.x) * inv.x;
    double t0y = (lo[1] - o.y) * inv.y, t1y = (hi[1] - o.y) * inv.y;
    double t0z = (lo[2] - o.z) * inv.z, t1z = (hi[2] - o.z) * inv.z;
    if (inv.x < 0.0) { double t = t0x; t0x = t1x; t1x = t; }
    if (inv.y < 0.0) { double t = t0y; t0y = t1y; t1y = t; }
    if (inv.z < 0.0) { double t = t0z; t0z = t1z; t1z = t; }
    double a = fmax(fmax(fmax(tmin, t0x), t0y), t0z);
    double b = fmin(fmin(fmin(tmax, t1x), t1y), t1z);
    entry = a;
    return !(b <= a);
}

// Test one leaf object with the range [tmin, best); on acceptance best := its t1 (the
// reference's right subtree is searched with `start..left.t1`, bvh.rs:179-188, i.e. the last
// accepted hit sets the range end, which is the minimum except for Difference's back-face hits).
template <bool SO>
__device__ __forceinline__ void test_leaf(const DScene& S, int p, const Ray& r, double tmin, double& best, double& bend,
                                          int& bp) {
    const DPrim P = S.prims[p];
    if (SO || P.kind == PK_SPHERE) {
        double t, t2;
        if (sphere_t(S.spheres[P.idx], r, tmin, best, t, t2)) { bend = best; best = t; bp = p; }
    } else {
        Hit tmp;
        if (Obj<RS_MAX_NEST>::hit(S, p, r, tmin, best, tmp)) { bend = best; best = tmp.t1; bp = p; }
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
// stk: this thread's column of the block's LDS stack (stride kBlock).
template <bool SO>
__device__ bool world_hit(const DScene& S, const Ray& r, double tmin, Hit& h, int* stk) {
    if (S.root < 0) return false;
    const V3 inv = v3(1.0 / r.d.x, 1.0 / r.d.y, 1.0 / r.d.z);
    double best = RS_INF, bend = RS_INF;
    int bp = -1;
    int node = S.root;
    int sp = 0;
    if (SO || !S.ref_order) {
        while (true) {
            const DNode& N = S.nodes[node];
            double e0, e1;
            const int c0 = N.child[0], c1 = N.child[1];
            bool h0 = slab(N.lo[0], N.hi[0], r.o, inv, tmin, best, e0);
            if (h0 && c0 < 0) { h0 = false; test_leaf<SO>(S, ~c0, r, tmin, best, bend, bp); }
            bool h1 = slab(N.lo[1], N.hi[1], r.o, inv, tmin, best, e1);
            if (h1 && c1 < 0) { h1 = false; if (c1 != INT32_MIN) test_leaf<SO>(S, ~c1, r, tmin, best, bend, bp); }
            if (h0 && h1) {
                int nn = c0, ff = c1;
                if (e1 < e0) { nn = c1; ff = c0; }
                stk[sp * kBlock] = ff;
                ++sp;
                node = nn;
            } else if (h0) {
                node = c0;
            } else if (h1) {
                node = c1;
            } else {
                if (sp == 0) break;
                --sp;
                node = stk[sp * kBlock];
            }
        }
    } else {
        bool second = false;  // visiting node's right child (left one already done)
        while (true) {
            const DNode& N = S.nodes[node];
            double e;
            if (!second) {
                const int c0 = N.child[0];
                if (slab(N.lo[0], N.hi[0], r.o, inv, tmin, best, e)) {
                    if (c0 < 0) {
                        test_leaf<SO>(S, ~c0, r, tmin, best, bend, bp);
                    } else {
                        stk[sp * kBlock] = node;  // come back for the right child
                        ++sp;
                        node = c0;
                        continue;
                    }
                }
            }
            const int c1 = N.child[1];
            if (c1 != INT32_MIN && slab(N.lo[1], N.hi[1], r.o, inv, tmin, best, e)) {
                if (c1 < 0) {
                    test_leaf<SO>(S, ~c1, r, tmin, best, bend, bp);
                } else {
                    node = c1;
                    second = false;
                    continue;
                }
            }
            if (sp == 0) break;
            --sp;
            node = stk[sp * kBlock];
            second = true;
        }
    }
    if (bp < 0) return false;
    // Recompute the full record of the winner with the exact range it was accepted under.
    if (SO || S.prims[bp].kind == PK_SPHERE) {
        const DPrim P = S.prims[bp];
        return sphere_hit(S.spheres[P.idx], P.mat, r, tmin, bend, h);
    }
    return Obj<RS_MAX_NEST>::hit(S, bp, r, tmin, bend, h);
}

// camera.rs:94-100
__device__ __forceinline__ double phong_highlight(V3 dir_to_light, V3 ray_dir, V3 n, int exponent, double factor) {
    V3 reflected = dir_to_light - (2.0 * dot(dir_to_light, n)) * n;
    double spec = powi_rt(fmax(dot(reflected, -ray_dir), 0.0), exponent);
    return spec * factor;
}

// TakePhotoSettings::ray_color (camera.rs:156-255), recursion unrolled into a loop with a
// running throughput. Returns the radiance of one camera sample.
template <bool SO>
__device__ V3 trace_path(const DScene& S, Ray ray, uint32_t depth, Rng& rng, int* stk, uint32_t& segs) {
    V3 T = v3(1.0, 1.0, 1.0);
    V3 L = v3(0.0, 0.0, 0.0);
    for (uint32_t d = depth; d > 0; --d) {
        ++segs;
        Hit h;
        if (!world_hit<SO>(S, ray, 0.0001, h, stk)) {
            V3 bg = background(S, ray);
            L = L + v3(T.x * bg.x, T.y * bg.y, T.z * bg.z);
            break;
        }
        const int mi = h.mat >= 0 ? h.mat : S.default_mat;
        const DMaterial& M0 = S.mats[mi];
        if (M0.kind == RS_MAT_DIFFUSE_LIGHT) {  // light.rs:33-35, scatter None
            float c[3];
            tex_color(M0, h.p, c);
            V3 e = v3((double)c[0] * M0.multiplier, (double)c[1] * M0.multiplier, (double)c[2] * M0.multiplier);
            L = L + v3(T.x * e.x, T.y * e.y, T.z * e.z);
            break;
        }
        int ms = mi;
        for (int k = 0; k < 16 && S.mats[ms].kind == RS_MAT_MIXED; ++k) {  // mixed_material.rs:43-50
            const DMaterial& X = S.mats[ms];
            ms = ((double)rng.next_u32() < 4294967295.0 * X.mix_p) ? X.mix_a : X.mix_b;
        }
        const DMaterial& M = S.mats[ms];
        float c[3];
        Pdf pdf;
        if (M.kind == RS_MAT_METAL) {  // metal.rs:104-118
            tex_color(M, h.p, c);
            V3 rf = reflect_v(ray.d, h.n);
            if (!(dot(rf, h.n) > 0.0)) break;
            T = v3(T.x * (double)c[0], T.y * (double)c[1], T.z * (double)c[2]);
            ray.o = h.p; ray.d = rf;
            continue;
        } else if (M.kind == RS_MAT_DIELECTRIC) {  // dielectric.rs:55-93
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
            continue;
        } else if (M.kind == RS_MAT_LAMBERTIAN) {  // lambertian.rs:39-50
            tex_color(M, h.p, c);
            pdf.kind = 0;
            pdf.n = onb_from(h.n);
        } else if (M.kind == RS_MAT_DIFFUSE_METAL) {  // metal.rs:54-68
            tex_color(M, h.p, c);
            V3 rf = reflect_v(ray.d, h.n);
            if (!(dot(rf, h.n) > 0.0)) break;
            pdf.kind = 1;
            pdf.exponent = M.exponent;
            pdf.refl = onb_from(reflect_v(ray.d, h.n));
            pdf.n = onb_from(h.n);
        } else {
            break;  // DiffuseLight reached through MixedMaterial: scatter None, no emission
        }
        // non-skip_pdf branch (camera.rs:194-247)
        double light_multi = 1.0, pdf_val;
        Ray nr;
        nr.time = ray.time;
        if (rng.gen() < 0.5) {
            pdf_val = 0.3183098861837907;
            const uint32_t li = rng.next_u32() % (uint32_t)S.n_lights;  // list.rs:49-52
            V3 rv;
            if (SO) rv = Obj<0>::sphere_random(S.spheres[S.prims[S.lights[li]].idx], h.p, rng);
            else rv = Obj<RS_MAX_NEST>::random(S, S.lights[li], h.p, rng);
            V3 dl = unit(rv);
            if (M0.phong_factor > 0.0)
                light_multi += phong_highlight(-dl, ray.d, h.n, M0.phong_exponent, M0.phong_factor);
            nr.o = ray_at(ray, h.t1 - 0.0002);
            nr.d = dl;
        } else {
            V3 sd = pdf_generate(pdf, rng);
            pdf_val = pdf_value(pdf, sd);
            nr.o = h.p;
            nr.d = sd;
        }
        if (pdf_val <= 0.0 || pdf_val != pdf_val) pdf_val = 1e-5;
        const double mult = pdf_value(pdf, nr.d) / pdf_val;
        T = v3(((double)c[0] * (light_multi * T.x)) * mult, ((double)c[1] * (light_multi * T.y)) * mult,
               ((double)c[2] * (light_multi * T.z)) * mult);
        ray = nr;
    }
    return L;
}

template <bool SO>
__global__ __launch_bounds__(kBlock) void k_path_mega(DScene S, DCamera C, PathParams P, double* __restrict__ rad,
                                                      unsigned long long* __restrict__ seg_counters) {
    __shared__ int stk_all[kStackMax * kBlock];
    int* stk = stk_all + threadIdx.x;
    const uint64_t item = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    uint32_t segs = 0;
    if (item < P.n_items) {
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
            L = trace_path<SO>(S, r, P.depth, rng, stk, segs);
        }
        rad[item] = L.x;
        rad[P.n_items + item] = L.y;
        rad[2 * P.n_items + item] = L.z;
    }
    // wave-reduce the segment count, one atomic per wave, spread over 256 counters
    unsigned long long s64 = segs;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s64 += __shfl_xor(s64, off, 64);
    if ((threadIdx.x & 63) == 0 && s64) atomicAdd(&seg_counters[blockIdx.x & 255], s64);
}

__global__ __launch_bounds__(kBlock) void k_accumulate(const double* __restrict__ rad, double* __restrict__ acc, uint32_t n_pix,
                                                      uint32_t n_samp, int first) {
    const uint32_t p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= n_pix) return;
    const uint64_t n_items = (uint64_t)n_pix * n_samp;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        double a = first ? 0.0 : acc[(uint64_t)c * n_pix + p];
        const double* rc = rad + (uint64_t)c * n_items + p;
        for (uint32_t s = 0; s < n_samp; ++s) a = a + rc[(uint64_t)s * n_pix];
        acc[(uint64_t)c * n_pix + p] = a;
    }
}

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

// Diagnostic: World::hit for a batch of rays (tests/ per-primitive parity probes).
// rays[i] = o(3) d(3) time; out[i] = hit t1 t2 p(3) n(3) 0 0 outside mat  (13 doubles, oracle layout)
__global__ __launch_bounds__(kBlock) void k_probe_hit(DScene S, const double* __restrict__ rays, uint32_t n, double tmin,
                                                     double tmax, double* __restrict__ out) {
    __shared__ int stk_all[kStackMax * kBlock];
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    Ray r;
    r.o = ld3(rays + 7 * i); r.d = ld3(rays + 7 * i + 3); r.time = rays[7 * i + 6];
    Hit h;
    double* o = out + 13 * (size_t)i;
    for (int k = 0; k < 13; ++k) o[k] = 0.0;
    // range end handled by clamping best: world_hit starts from +inf, so emulate [tmin, tmax) by a
    // post-check only when tmax is infinite (the render path always passes +inf)
    if (world_hit<false>(S, r, tmin, h, stk_all + threadIdx.x) && h.t1 < tmax) {
        o[0] = 1.0; o[1] = h.t1; o[2] = h.t2;
        o[3] = h.p.x; o[4] = h.p.y; o[5] = h.p.z; o[6] = h.n.x; o[7] = h.n.y; o[8] = h.n.z;
        o[11] = h.outside ? 1.0 : 0.0; o[12] = (double)h.mat;
    }
}

hipError_t launch_probe_hit(const DScene& s, const double* rays, uint32_t n, double tmin, double tmax, double* out,
                            hipStream_t st) {
    const uint32_t blocks = (n + kBlock - 1) / kBlock;
    if (!blocks) return hipSuccess;
    hipLaunchKernelGGL(k_probe_hit, dim3(blocks), dim3(kBlock), 0, st, s, rays, n, tmin, tmax, out);
    return hipGetLastError();
}

hipError_t launch_path_mega(const DScene& s, const DCamera& c, const PathParams& p, bool spheres_only, double* rad,
                            unsigned long long* seg_counters, hipStream_t st) {
    const uint64_t blocks = (p.n_items + kBlock - 1) / kBlock;
    if (blocks == 0) return hipSuccess;
    if (spheres_only)
        hipLaunchKernelGGL(k_path_mega<true>, dim3((uint32_t)blocks), dim3(kBlock), 0, st, s, c, p, rad, seg_counters);
    else
        hipLaunchKernelGGL(k_path_mega<false>, dim3((uint32_t)blocks), dim3(kBlock), 0, st, s, c, p, rad, seg_counters);
    return hipGetLastError();
}

hipError_t launch_accumulate(const double* rad, double* acc, uint32_t n_pix, uint32_t n_samp_batch, int first_batch,
                             hipStream_t st) {
    const uint32_t blocks = (n_pix + kBlock - 1) / kBlock;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_accumulate, dim3(blocks), dim3(kBlock), 0, st, rad, acc, n_pix, n_samp_batch, first_batch);
    return hipGetLastError();
}

hipError_t launch_finalize(const double* acc, float* out_rgba, const FinalParams& p, hipStream_t st) {
    const uint32_t blocks = (p.n_pix_local + kBlock - 1) / kBlock;
    if (blocks == 0) return hipSuccess;
    hipLaunchKernelGGL(k_finalize, dim3(blocks), dim3(kBlock), 0, st, acc, out_rgba, p);
    return hipGetLastError();
}

}  // namespace rs
