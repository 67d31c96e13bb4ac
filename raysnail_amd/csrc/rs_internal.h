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
// the smallest LDS part of any path kernel (stack_lds below): the overflow array is sized for it, so
// every kernel that walks a scene fits it
constexpr int kStackMin = 16;
// leaves listed per walk by the deferred reference-order traversal (LDS-image scenes), in the top
// kLeafBatch entries of the thread's LDS stack column
constexpr uint32_t kLeafBatch = 8;
constexpr uint32_t kMaxLanes = 4;   // chunk lanes of the bounce-synchronous wavefront (flat / rich scenes)
constexpr uint32_t kMaxSlots = 4;   // frames in flight per replica (rs_scene_set_frames_in_flight)

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
// the streaming (material-sorted) wavefront serves these modes; flat (mesh) and generic scenes run
// the bounce-synchronous unsorted wavefront
constexpr bool streaming_mode(int sm) { return sm == kSmSpheres || sm == kSmNest0 || sm == kSmNest2; }
// LDS stack entries per thread of the path kernels (k_wf_extend, k_wfs_extend) by scene mode: 16, 24 in the
// rich mode. A 32 KiB block (24 entries + the mesh extend's 8-entry leaf FIFO) kept only 4 of the flat extend's
// 5 blocks per CU resident; at 16 entries the C5 mesh frame is 10 % faster although more of its deep entries
// spill to HBM, C4 2.5 % and example.sdl 1.6 %; the rich mode (X2) lost 4 % (profiles/r4/ab/lds_stack). The
// spheres mode takes 16 since round 5: its extend's LDS tree top (kLTop) then fits 5 blocks per CU.
constexpr int stack_lds(int sm) { return sm == kSmGeneric ? kStackMax : kStackMin; }
// the nest modes' LDS scene image (rs_layout.h kLimgMax) next to their stack: four 256-thread blocks per CU
// must fit the CU's 160 KiB of LDS
static_assert(4u * ((uint32_t)stack_lds(kSmNest0) * kBlock * 4u + kLimgMax) <= 160u * 1024u, "LDS image budget");
static_assert(4u * ((uint32_t)stack_lds(kSmNest2) * kBlock * 4u + kLimgMax) <= 160u * 1024u, "LDS image budget");

// A committed scene for a launch: the host copy (launch decisions) and the same struct in device
// memory, which the kernels read through a pointer (a by-value kernel argument that device functions
// take by reference is copied to scratch).
struct SceneRef {
    const DScene* host;
    const DScene* dev;
};
// flat scenes on the 4-wide tree: the persistent extend with lane refill (k_wf_extend_dyn; RS_NO_FLAT_DYN: the
// one-ray-per-lane k_wf_extend, for A/B)
#if defined(RS_NO_FLAT_DYN) || defined(RS_TRAV_STATS)
inline bool flat_dyn(const SceneRef&) { return false; }
#else
inline bool flat_dyn(const SceneRef& s) { return s.host->root4 >= 0; }
#endif
// flat scenes whose shading is Lambertian / DiffuseLight only: k_wf_shade<kSmFlat, true> (RS_NO_FLAT_LAMB: the
// generic one, for A/B)
#ifdef RS_NO_FLAT_LAMB
inline bool flat_lamb(const SceneRef&) { return false; }
#else
inline bool flat_lamb(const SceneRef& s) { return s.host->lamb_only != 0; }
#endif

// The frame's camera-sample lattice: item = sample * n_pix_local + lattice pixel (painter.rs:154-187
// per pixel, render_rows' row interleave painter.rs:248 per lattice row).
struct PathParams {
    uint64_t n_items;
    uint32_t n_pix_local;   // pixels on the row lattice
    uint32_t width, height;
    uint32_t row_begin, row_step;
    uint32_t sqrt_spp;
    uint32_t s0;            // first sample index of the batch (bounce-synchronous wavefront, megakernel)
    uint32_t depth;
    uint64_t key_base;      // splitmix64(splitmix64(seed) ^ pass)
    const uint8_t* mask;    // device, W*H or null
};

// 32-byte path-state record (one wave load = 2 KiB contiguous)
struct alignas(32) D4 { double x, y, z, w; };
// A material-class queue entry of the streaming wavefront: the path's record slot in the current set and its
// World::hit result (the winning prim; in the spheres mode the winner's t, otherwise the range end it was accepted
// under), 16 bytes written by the extend in queue order, so the shading reads its batch's entries contiguously
// instead of gathering the hit by record slot (a sparse class's 16-byte hit gather took a 128-byte line each)
struct alignas(16) QEnt {
    uint32_t i;
    int32_t bp;
    double t;
};

// Wavefront path state. 32-byte records per path per array, in two ping-pong sets: a launch reads
// set t&1 and the survivors are written, compacted, into set (t+1)&1, so every kernel streams
// contiguous records. The XorShift128 state rides in the fourth lanes of ray_d / thr (as bits). A
// live path's radiance is not stored: it is always 0 (ray_color adds emission / background only
// where the recursion ends, camera.rs:172-254), so a path's result is 0 + T * (its last term).
struct WfSet {
    D4* ray_o;            // origin xyz + time
    D4* ray_d;            // direction xyz + rng (x | y << 32)
    D4* thr;              // throughput xyz + rng (z | w << 32)
    uint2* tag;           // x: the path's radiance slot (its camera sample's rad index); y: its ray_color
                          // level (segments traced: the streaming wavefront's depth limit) -- one 8-byte
                          // load where the shading gathers them
};
struct WfState {
    WfSet set[2];
    double2* hit;         // bounce-synchronous wavefront, per slot of the current set: (prim as bits, accepted range
                          // end) -- the memory of the class queues, which only the streaming wavefront uses
    uint32_t* counts;     // counter block per launch step (stride kWfsStride / 1 words)
    uint32_t* fetch;      // k_wf_extend_dyn's chunk counters (flat scenes)
    uint32_t* heads;      // bounce-synchronous sets: 2 banks x 8 shards x (count, region offset) (rs_kernels.hip Segs)
    uint32_t cap;         // records per set (the sorted path fills a set from both ends)
    uint32_t tagw;        // 1: no moving sphere -- (item, level) ride in ray_o.w instead of `tag` (rs_kernels.hip store_path)
};

// Streaming wavefront (k_wfs_extend): the camera samples injected by one iteration. The frame's
// samples are injected in gen_perm order batch by batch (a batch = whole sample planes of the row
// lattice, `batch` items); an iteration injects at most `batch` samples, so it crosses at most one
// batch boundary. Batch k's radiance goes to the rad ring's buffer k % ring_batches (k_accumulate
// empties a buffer, in sample order, once every sample of its batch has finished).
struct InjParams {
    uint32_t n_new;       // camera samples injected by this iteration
    uint32_t jb0;         // the first one's index inside its batch (gen_perm order)
    uint32_t nb0;         // items in that batch
    uint32_t nb1;         // items in the next batch (0: none)
    uint64_t g0, g1;      // frame items of the two batches' starts (k * batch: a lane's batches are not adjacent)
    uint32_t rad0, rad1;  // rad ring offsets of the two batches' buffers
    uint64_t key0, key1;  // the two batches' PathParams::key_base (a multi-pass stream: their passes' keys)
};

struct FinalParams {
    uint32_t n_pix_local, width, row_begin, row_step;
    uint32_t n_samples;
    int32_t gamma;
    const uint8_t* mask;
};

// Megakernel: one thread per (pixel, sample) path (grid-stride over at most max_blocks blocks);
// radiance -> rad[3 * item + c] (item-major, rs_kernels.hip put_rad, like every path kernel).
hipError_t launch_probe_sample(const SceneRef& s, const DCamera& c, const PathParams& p, int sm, uint32_t x, uint32_t y,
                               uint32_t s0, uint32_t n, double* out, hipStream_t st);
hipError_t launch_path_mega(const SceneRef& s, const DCamera& c, const PathParams& p, int sm, double* rad,
                            unsigned long long* seg_counters, uint32_t max_blocks, hipStream_t st);
// bounce-synchronous unsorted wavefront (flat / rich scenes): camera rays of a chunk, then per bounce
// extend + shade
hipError_t launch_wf_gen(const DCamera& c, const PathParams& p, const WfState& w, uint64_t item0, uint32_t n, double* rad,
                         hipStream_t st);
hipError_t launch_wf_extend(const SceneRef& s, const WfState& w, uint32_t bounce, uint32_t blocks, int sm, hipStream_t st);
hipError_t launch_wf_shade(const SceneRef& s, const WfState& w, uint32_t bounce, uint32_t depth, uint64_t n_items, double* rad,
                           uint32_t blocks, int sm, hipStream_t st);

constexpr int kWfsClasses = 5;   // Lambertian, Metal, DiffuseMetal, Dielectric, other
#ifndef RS_CNT_PAD
#define RS_CNT_PAD 32  // counters 128 B apart: one line each, so the block-aggregated atomics of
                       // different classes do not serialise on one L2 line (bench frame 9.89 -> 9.58 ms)
#endif
constexpr uint32_t kCntPad = RS_CNT_PAD;
// counter slots per streaming iteration: 0 paths carried in from the previous iteration, 1-5 class
// queues, 6 / 7 front / back runs of the next set, 8 .. 8 + kStatLines - 1 the iteration's live
// camera samples spread over lines by block (a single word takes only ~88 atomics/us; summed by the
// host; the iteration's segments are slot 0 + these)
constexpr int kCntStat0 = 8;
constexpr uint32_t kStatLines = 8;
constexpr uint32_t kWfsStride = (kCntStat0 + kStatLines) * kCntPad;
// word index of counter `slot` in an iteration's block
__host__ __device__ constexpr uint32_t cix(int slot) { return (uint32_t)slot * kCntPad; }
// counts[6] / counts[7]: paths written from the front / the back of the next set (light-sample rays
// / the rest), so the next extend's waves hold rays of one kind; the injected camera rays go between
constexpr int kCntFront = 6, kCntBack = 7;
// Streaming iteration `it`: extend every path carried in (set it&1, front and back runs) plus the
// iteration's injected camera samples; class queues in counter block `it`. part: 0 both in one launch,
// 1 the carried paths, 2 the camera samples (ext_split: two launches per iteration). ev0 / ev1 (may be
// null): start / stop events carried by the dispatch itself (hipExtLaunchKernel: no separate packets).
constexpr int kExtAll = 0, kExtCarried = 1, kExtCamera = 2;
// nest-2 scenes extend in two launches: the merged kernel needs 256 VGPRs + 2 AGPRs (one wave/SIMD); the spheres
// mode too since its carried launches take grids from the last frame's counts (rs_host.cpp Replica::hist) and its
// carried part runs at 5 waves: a C3-shaped frame (1920x1080x64, depth 50) 42.4 -> 41.1 ms
// (profiles/r6/ab/ext_split_spheres_r6h5.jsonl; nest-0 example.sdl equal, so it keeps the merged launch)
constexpr bool ext_split(int sm) { return sm == kSmNest2 || sm == kSmSpheres; }
hipError_t launch_wfs_extend(const SceneRef& s, const DCamera& c, const PathParams& p, const WfState& w,
                             QEnt* const* queues, uint32_t it, const InjParams& inj, double* rad, uint32_t blocks,
                             int part, int sm, hipStream_t st, hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
// every material class of iteration `it` in one launch (k_wfs_shade_all); class_mask: classes present
// the streaming frame's last iteration: every carried path of set it&1 traced to its end, one thread each
// (k_wfs_finish); blocks: at least one per 256 carried paths (grid-stride)
hipError_t launch_wfs_finish(const SceneRef& s, const WfState& w, uint32_t it, uint32_t depth, double* rad, uint32_t blocks,
                             int sm, hipStream_t st);
// split: the spheres mode's lean and heavy material classes in two launches (k_wfs_shade_all PS)
hipError_t launch_wfs_shade_all(const SceneRef& s, const WfState& w, QEnt* const* queues, uint32_t class_mask,
                                uint32_t it, uint32_t depth, double* rad, uint32_t blocks, bool split, int sm,
                                hipStream_t st);
// blocks per CU the extend / shade kernels can keep resident (occupancy API), for grid-stride grids
hipError_t wf_occupancy(int sm, int* extend_blocks_per_cu, int* shade_blocks_per_cu);
hipError_t launch_combine(float* acc, const float* nw, uint64_t n, float p, hipStream_t st);
hipError_t launch_noise(const float* px, int w, int h, float t, uint8_t* redo, unsigned int* minmax_bits,
                        unsigned long long* count, hipStream_t st);
hipError_t launch_probe_hit(const SceneRef& s, const double* rays, uint32_t n, double tmin, double tmax, double* out,
                            hipStream_t st);
// acc[c * n_pix + pixel] += sum over the batch's samples in sample order (deterministic; item-major
// radiance rad[3 * item + c], items sample-plane by sample-plane); the last batch writes into_color of the sum into the frame instead (k_finalize's
// arithmetic, one launch less) and zeroes zero[0, n_zero) (the frame's queue counters) for the next
// frame.
hipError_t launch_accumulate(const double* rad, double* acc, uint32_t n_pix, uint32_t n_samp_batch,
                             int first_batch, int last_batch, const FinalParams& p, float* out_rgba, uint32_t* zero,
                             uint32_t n_zero, hipStream_t st);
// into_color + RGBA f32 store into the full frame.
hipError_t launch_finalize(const double* acc, float* out_rgba, const FinalParams& p, hipStream_t st);

}  // namespace rs
