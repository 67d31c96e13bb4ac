// rs_internal.h — host <-> kernel launch interface (not part of the public ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "rs_layout.h"

namespace rs {

constexpr int kBlock = 256;      // 4 waves of 64
// per-thread BVH stack entries held in LDS (24 KiB/block -> 6 blocks/CU); deeper entries spill to
// DScene::stk_ovf, which the host sizes from the tree's exact worst-case stack depth
constexpr int kStackMax = 24;
#ifndef RS_LANES
#define RS_LANES 2  // wavefront lanes: chunks of a batch in flight together on this many streams
#endif
constexpr uint32_t kMaxLanes = 4;
#ifndef RS_PH_N
#define RS_PH_N 0     // phased flat-scene extend: bounded phases by default (RS_PHASES overrides)
#endif
#ifndef RS_PH_B0
#define RS_PH_B0 24   // node-step budget of phase 0
#endif
#ifndef RS_PH_B1
#define RS_PH_B1 16
#endif


// One batch of camera samples: items = n_pix_local * n_samp_batch, item -> (sample, pixel).
// Scene modes (a template parameter of every path kernel): kSmSpheres -- world and lights are
// spheres only (prim-indexed sphere copy, material-sorted wavefront); kSmFlat -- spheres, rects and
// triangles only (no CSG / transforms / boxes / quadrics: leaf tests without the nested object
// machinery); kSmNest0 / kSmNest2 -- anything with at most 0 / 2 levels of CSG / TfFacade nesting
// (the nested-object code is instantiated only as deep as the scene needs: fewer registers, no
// scratch); kSmGeneric -- up to RS_MAX_NEST levels.
enum SceneMode { kSmGeneric = 0, kSmSpheres = 1, kSmFlat = 2, kSmNest0 = 3, kSmNest2 = 4 };
constexpr int nest_of(int sm) { return sm == kSmNest0 ? 0 : sm == kSmNest2 ? 2 : sm == kSmGeneric ? RS_MAX_NEST : 0; }
// the generic mode is also the rich one: ConstantMedium, Perlin / Image textures, (u, v) records
// (commit puts every scene that uses them there; the other modes compile none of that code)
constexpr int rich_of(int sm) { return sm == kSmGeneric ? 1 : 0; }

// A committed scene for a launch: the host copy (launch decisions) and the same struct in device
// memory, which the kernels read through a pointer (a by-value kernel argument that device functions
// take by reference is copied to scratch).
struct SceneRef {
    const DScene* host;
    const DScene* dev;
};

struct PathParams {
    uint64_t n_items;
    uint32_t n_pix_local;   // pixels on the row lattice
    uint32_t width, height;
    uint32_t row_begin, row_step;
    uint32_t sqrt_spp;
    uint32_t s0;            // first sample index of the batch
    uint32_t depth;
    uint64_t key_base;      // splitmix64(splitmix64(seed) ^ pass)
    const uint8_t* mask;    // device, W*H or null
};

// 32-byte path-state record (one wave load = 2 KiB contiguous)
struct alignas(32) D4 { double x, y, z, w; };

// Wavefront path state (capacity = chunk size). 32-byte records per path per array, in two
// ping-pong sets: bounce b reads set b&1 at [0, counts[b]) and the survivors are written,
// compacted, into set (b+1)&1, so every kernel streams contiguous records. The XorShift128 state
// rides in the fourth lanes of ray_d / thr (as bits). A live path's radiance is not stored: it is
// always 0 (ray_color adds emission / background only where the recursion ends, camera.rs:172-254),
// so a path's result is 0 + T * (its last term). 100 bytes per path and set.
struct WfSet {
    D4* ray_o;            // origin xyz + time
    D4* ray_d;            // direction xyz + rng (x | y << 32)
    D4* thr;              // throughput xyz + rng (z | w << 32)
    uint32_t* item;       // batch item (sample, pixel) of the path
};
struct WfState {
    WfSet set[2];
    double2* hit;         // per compacted slot of the current bounce: (prim as bits, accepted range end)
    uint32_t* counts;     // [depth + 1] live paths per bounce
    uint32_t cap;         // records per set (the sorted path fills a set from both ends, see k_wfs_shade)
    uint32_t qsub;        // records per class sub-queue (qsub_cap(cap))
};

struct FinalParams {
    uint32_t n_pix_local, width, row_begin, row_step;
    uint32_t n_samples;
    int32_t gamma;
    const uint8_t* mask;
};

// Megakernel: one thread per (pixel, sample) path (grid-stride over at most max_blocks blocks);
// radiance -> rad[c * n_items + item].
hipError_t launch_probe_sample(const SceneRef& s, const DCamera& c, const PathParams& p, int sm, uint32_t x, uint32_t y,
                               uint32_t s0, uint32_t n, double* out, hipStream_t st);
hipError_t launch_path_mega(const SceneRef& s, const DCamera& c, const PathParams& p, int sm, double* rad,
                            unsigned long long* seg_counters, uint32_t max_blocks, hipStream_t st);
hipError_t launch_wf_gen(const DCamera& c, const PathParams& p, const WfState& w, uint64_t item0, uint32_t n, double* rad,
                         hipStream_t st);
hipError_t launch_wf_extend(const SceneRef& s, const WfState& w, uint32_t bounce, uint32_t blocks, int sm, hipStream_t st);
hipError_t launch_wf_shade(const SceneRef& s, const WfState& w, uint32_t bounce, uint32_t depth, uint64_t n_items, double* rad,
                           uint32_t blocks, int sm, hipStream_t st);
// Suspended traversals of the phased flat-scene extend (k_wf_extend_ph), SoA over cap slots: the
// path's slot in the bounce's set, the next node, stack depth, best leaf entry, range end and the
// accepted range end; stack entry k of slot j at stk[k * cap + j].
struct ContSet {
    uint32_t* idx;
    int32_t* node;
    int32_t* sp;
    int32_t* bp;
    double* best;
    double* bend;
    int32_t* stk;
    uint32_t cap;
};
constexpr int kMaxPhases = 4;
// One phase of a flat scene's extend at `bounce`: in_cnt == nullptr starts every path of the bounce,
// otherwise the in_cnt suspended traversals of `in` are resumed; each runs at most `budget` node
// steps (budget < 0: to the end) and the ones still open are appended to `out` / out_cnt.
hipError_t launch_wf_extend_ph(const SceneRef& s, const WfState& w, uint32_t bounce, const ContSet& in,
                               const uint32_t* in_cnt, const ContSet& out, uint32_t* out_cnt, int budget, uint32_t blocks,
                               hipStream_t st);
// material-sorted variant (every scene mode but the generic / rich one): counts stride per bounce = kWfsStride
#ifndef RS_SORTED_FLAT
#define RS_SORTED_FLAT 0  // flat scenes (meshes) on the material-sorted wavefront too
#endif
constexpr int kWfsClasses = 5;   // Lambertian, Metal, DiffuseMetal, Dielectric, other
#ifndef RS_CNT_PAD
#define RS_CNT_PAD 32  // queue counters 128 B apart: one line each, so the block-aggregated atomics of
                       // different classes do not serialise on one L2 line (bench frame 9.89 -> 9.58 ms)
#endif
constexpr uint32_t kCntPad = RS_CNT_PAD;
// Each class queue is split into kQSub sub-queues with a counter each: batch q of 256 paths of an
// extend launch appends to sub-queue q % kQSub, so the block-aggregated atomics spread over kQSub
// lines per class instead of serialising on one. A sub-queue holds at most WfState::qsub records
// (the batches q == g mod kQSub of a set), the shading kernels walk the sub-queues in order.
#ifndef RS_QSUB
#define RS_QSUB 1  // measured: 4, 8, 16 sub-queues are slower (bench frame 9.06 -> 9.18, 9.25, 9.39 ms)
#endif
constexpr uint32_t kQSub = RS_QSUB;
// slots per bounce: 0 live paths, 1-5 class queues, 6 / 7 front / back runs of the next set,
// 8 .. 8 + kStatLines - 1 the bounce-0 live-sample count spread over lines (summed by the host)
constexpr int kCntStat0 = 8;
constexpr uint32_t kStatLines = 8;
constexpr uint32_t kWfsStride = (8 + kStatLines) * kQSub * kCntPad;
// word index of counter `slot` (0 live, 1 + k class k, kCntFront, kCntBack), sub-counter g, in a bounce's block
__host__ __device__ constexpr uint32_t cix(int slot, uint32_t g = 0) { return ((uint32_t)slot * kQSub + g) * kCntPad; }
__host__ __device__ constexpr uint32_t qsub_cap(uint32_t cap) {
    return ((cap + 255u) / 256u + kQSub - 1u) / kQSub * 256u;
}
// counts[6] / counts[7] of a bounce: paths written from the front / the back of the set (light-
// sample rays / the rest), so the next extend's waves hold rays of one kind (k_wfs_shade)
constexpr int kCntFront = 6, kCntBack = 7;
#ifndef RS_SHADE_MERGED
#define RS_SHADE_MERGED 1  // shading launches per bounce: 0 one per class; 1 classes 0-3 merged; 2 classes 1-3 merged
#endif
constexpr int kShadeAllFirst = RS_SHADE_MERGED == 2 ? 1 : 0;
// ev0 / ev1 (may be null): start / stop events carried by the dispatch itself (hipExtLaunchKernel:
// no separate event packets, so timing adds no gap between kernels)
hipError_t launch_wfs_gen_extend(const SceneRef& s, const DCamera& c, const PathParams& p, const WfState& w,
                                uint32_t* const* queues, uint32_t stride, uint64_t item0, uint32_t n, double* rad,
                                uint32_t blocks, int sm, hipStream_t st, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
hipError_t launch_wfs_extend(const SceneRef& s, const WfState& w, uint32_t* const* queues, uint32_t bounce, uint32_t stride,
                            uint64_t n_items, double* rad, uint32_t blocks, int sm, hipStream_t st,
                            hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
// every material class of bounce `bounce` in one launch (k_wfs_shade_all); class_mask: classes present
hipError_t launch_wfs_shade_all(const SceneRef& s, const WfState& w, uint32_t* const* queues, uint32_t class_mask,
                                uint32_t bounce, uint32_t stride, uint32_t depth, uint64_t n_items, double* rad,
                                uint32_t blocks, int sm, hipStream_t st);
hipError_t launch_wfs_shade(const SceneRef& s, const WfState& w, const uint32_t* queue, int cls, uint32_t bounce,
                           uint32_t stride, uint32_t depth, uint64_t n_items, double* rad, uint32_t blocks, int sm,
                           hipStream_t st);
// blocks per CU the extend / shade kernels can keep resident (occupancy API), for grid-stride grids
hipError_t wf_occupancy(int sm, int* extend_blocks_per_cu, int* shade_blocks_per_cu);
hipError_t launch_combine(float* acc, const float* nw, uint64_t n, float p, hipStream_t st);
hipError_t launch_noise(const float* px, int w, int h, float t, uint8_t* redo, unsigned int* minmax_bits,
                        unsigned long long* count, hipStream_t st);
hipError_t launch_probe_hit(const SceneRef& s, const double* rays, uint32_t n, double tmin, double tmax, double* out,
                            hipStream_t st);
// acc[c * n_pix + pixel] += sum over the batch's samples in sample order (deterministic); the last
// batch writes into_color of the sum into the frame instead (k_finalize's arithmetic, one launch less)
// and zeroes zero[0, n_zero) (the frame's queue counters) for the next frame.
hipError_t launch_accumulate(const double* rad, double* acc, uint32_t n_pix, uint32_t n_samp_batch, int first_batch,
                             int last_batch, const FinalParams& p, float* out_rgba, uint32_t* zero, uint32_t n_zero,
                             hipStream_t st);
// into_color + RGBA f32 store into the full frame.
hipError_t launch_finalize(const double* acc, float* out_rgba, const FinalParams& p, hipStream_t st);

}  // namespace rs
