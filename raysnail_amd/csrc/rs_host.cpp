// rs_host.cpp — host half of libraysnail_hip.so: the C-ABI (include/raysnail_hip.h), scene
// flattening into the device layout (rs_layout.h), bounding boxes, BVH build, upload and the
// render orchestration (batches of camera samples -> ordered accumulation -> into_color).
//
// Reference behaviour restated here (host side, once per scene / frame):
//   bounding boxes        sphere.rs:117-142, rect.rs:127-139, box.rs:155-157 (faces list.rs:68-81),
//                         quadric.rs:191-196, triangle_mesh.rs:133-135, intersection.rs:102-115
//                         (min.z from b1.min.y, kept), difference.rs:109-111, tf_facade.rs:58-90
//   transforms            transform.rs:16-107 (+ vecmath 1.0.0 mat4_inv)
//   Camera::new           camera.rs:37-73, CameraBuilder width/height aspect camera.rs:384-397
//   Painter::samples      painter.rs:110-118 (N = floor(sqrt(requested))^2)
// The BVH is this library's own (binned SAH, one object per leaf); BVH topology is not a parity
// obligation because every leaf box is the object's own bbox.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <functional>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <new>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/raysnail_hip.h"
#include "rs_internal.h"
#include "rs_layout.h"

using namespace rs;

namespace {

thread_local std::string g_last_error;

struct Error : std::runtime_error {
    int code;
    Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIP_OK(x)                                                                                          \
    do {                                                                                                   \
        hipError_t e_ = (x);                                                                               \
        if (e_ != hipSuccess) throw Error(RS_E_HIP, std::string(#x " failed: ") + hipGetErrorString(e_)); \
    } while (0)

struct Box3 {
    double lo[3], hi[3];
};
Box3 box_union(const Box3& a, const Box3& b) {
    Box3 r;
    for (int i = 0; i < 3; ++i) { r.lo[i] = std::fmin(a.lo[i], b.lo[i]); r.hi[i] = std::fmax(a.hi[i], b.hi[i]); }
    return r;
}
Box3 box_empty() {
    Box3 r;
    for (int i = 0; i < 3; ++i) { r.lo[i] = INFINITY; r.hi[i] = -INFINITY; }
    return r;
}

// host object record, one per handle
struct HObj {
    int32_t kind = 0;
    int32_t mat = RS_NO_MATERIAL;
    double p[18] = {0};
    int32_t a = -1, b = -1;            // children (CSG / XFORM child in a)
    int32_t ax[3] = {0, 0, 0};         // rect axes
    std::vector<rs_transform> tfs;     // XFORM
};

struct HPerlin {   // rs_perlin_desc with its tables copied
    rs_perlin_desc d;
    std::vector<double> values;
    std::vector<int32_t> perms;        // perm_x, perm_y, perm_z
};
struct HImage {
    uint32_t w = 0, h = 0;
    std::vector<uint8_t> rgb;
};

typedef double M4[4][4];

// vecmath 1.0.0 mat4_det / mat4_inv: explicit cofactor expansion, 1/det scaling.
double det4(const M4 m) {
    double pos = m[0][0] * m[1][1] * m[2][2] * m[3][3] + m[0][0] * m[1][2] * m[2][3] * m[3][1] +
                 m[0][0] * m[1][3] * m[2][1] * m[3][2] + m[0][1] * m[1][0] * m[2][3] * m[3][2] +
                 m[0][1] * m[1][2] * m[2][0] * m[3][3] + m[0][1] * m[1][3] * m[2][2] * m[3][0] +
                 m[0][2] * m[1][0] * m[2][1] * m[3][3] + m[0][2] * m[1][1] * m[2][3] * m[3][0] +
                 m[0][2] * m[1][3] * m[2][0] * m[3][1] + m[0][3] * m[1][0] * m[2][2] * m[3][1] +
                 m[0][3] * m[1][1] * m[2][0] * m[3][2] + m[0][3] * m[1][2] * m[2][1] * m[3][0];
    return pos - m[0][0] * m[1][1] * m[2][3] * m[3][2] - m[0][0] * m[1][2] * m[2][1] * m[3][3] -
           m[0][0] * m[1][3] * m[2][2] * m[3][1] - m[0][1] * m[1][0] * m[2][2] * m[3][3] -
           m[0][1] * m[1][2] * m[2][3] * m[3][0] - m[0][1] * m[1][3] * m[2][0] * m[3][2] -
           m[0][2] * m[1][0] * m[2][3] * m[3][1] - m[0][2] * m[1][1] * m[2][0] * m[3][3] -
           m[0][2] * m[1][3] * m[2][1] * m[3][0] - m[0][3] * m[1][0] * m[2][1] * m[3][2] -
           m[0][3] * m[1][1] * m[2][2] * m[3][0] - m[0][3] * m[1][2] * m[2][0] * m[3][1];
}
// cofactor term: sum of three "+" triple products minus three "-" ones, as vecmath writes them
double cof(const M4 m, int a0, int a1, int b0, int b1, int c0, int c1, int d0, int d1, int e0, int e1, int f0, int f1,
           int g0, int g1, int h0, int h1, int i0, int i1, int j0, int j1, int k0, int k1, int l0, int l1,
           int mm0, int mm1, int n0, int n1, int o0, int o1, int q0, int q1, int r0, int r1, int s0, int s1) {
    return m[a0][a1] * m[b0][b1] * m[c0][c1] + m[d0][d1] * m[e0][e1] * m[f0][f1] + m[g0][g1] * m[h0][h1] * m[i0][i1] -
           m[j0][j1] * m[k0][k1] * m[l0][l1] - m[mm0][mm1] * m[n0][n1] * m[o0][o1] - m[q0][q1] * m[r0][r1] * m[s0][s1];
}
void inv4(const M4 m, M4 o) {
    const double id = 1.0 / det4(m);
    o[0][0] = cof(m, 1,1,2,2,3,3, 1,2,2,3,3,1, 1,3,2,1,3,2, 1,1,2,3,3,2, 1,2,2,1,3,3, 1,3,2,2,3,1) * id;
    o[0][1] = cof(m, 0,1,2,3,3,2, 0,2,2,1,3,3, 0,3,2,2,3,1, 0,1,2,2,3,3, 0,2,2,3,3,1, 0,3,2,1,3,2) * id;
    o[0][2] = cof(m, 0,1,1,2,3,3, 0,2,1,3,3,1, 0,3,1,1,3,2, 0,1,1,3,3,2, 0,2,1,1,3,3, 0,3,1,2,3,1) * id;
    o[0][3] = cof(m, 0,1,1,3,2,2, 0,2,1,1,2,3, 0,3,1,2,2,1, 0,1,1,2,2,3, 0,2,1,3,2,1, 0,3,1,1,2,2) * id;
    o[1][0] = cof(m, 1,0,2,3,3,2, 1,2,2,0,3,3, 1,3,2,2,3,0, 1,0,2,2,3,3, 1,2,2,3,3,0, 1,3,2,0,3,2) * id;
    o[1][1] = cof(m, 0,0,2,2,3,3, 0,2,2,3,3,0, 0,3,2,0,3,2, 0,0,2,3,3,2, 0,2,2,0,3,3, 0,3,2,2,3,0) * id;
    o[1][2] = cof(m, 0,0,1,3,3,2, 0,2,1,0,3,3, 0,3,1,2,3,0, 0,0,1,2,3,3, 0,2,1,3,3,0, 0,3,1,0,3,2) * id;
    o[1][3] = cof(m, 0,0,1,2,2,3, 0,2,1,3,2,0, 0,3,1,0,2,2, 0,0,1,3,2,2, 0,2,1,0,2,3, 0,3,1,2,2,0) * id;
    o[2][0] = cof(m, 1,0,2,1,3,3, 1,1,2,3,3,0, 1,3,2,0,3,1, 1,0,2,3,3,1, 1,1,2,0,3,3, 1,3,2,1,3,0) * id;
    o[2][1] = cof(m, 0,0,2,3,3,1, 0,1,2,0,3,3, 0,3,2,1,3,0, 0,0,2,1,3,3, 0,1,2,3,3,0, 0,3,2,0,3,1) * id;
    o[2][2] = cof(m, 0,0,1,1,3,3, 0,1,1,3,3,0, 0,3,1,0,3,1, 0,0,1,3,3,1, 0,1,1,0,3,3, 0,3,1,1,3,0) * id;
    o[2][3] = cof(m, 0,0,1,3,2,1, 0,1,1,0,2,3, 0,3,1,1,2,0, 0,0,1,1,2,3, 0,1,1,3,2,0, 0,3,1,0,2,1) * id;
    o[3][0] = cof(m, 1,0,2,2,3,1, 1,1,2,0,3,2, 1,2,2,1,3,0, 1,0,2,1,3,2, 1,1,2,2,3,0, 1,2,2,0,3,1) * id;
    o[3][1] = cof(m, 0,0,2,1,3,2, 0,1,2,2,3,0, 0,2,2,0,3,1, 0,0,2,2,3,1, 0,1,2,0,3,2, 0,2,2,1,3,0) * id;
    o[3][2] = cof(m, 0,0,1,2,3,1, 0,1,1,0,3,2, 0,2,1,1,3,0, 0,0,1,1,3,2, 0,1,1,2,3,0, 0,2,1,0,3,1) * id;
    o[3][3] = cof(m, 0,0,1,1,2,2, 0,1,1,2,2,0, 0,2,1,0,2,1, 0,0,1,2,2,1, 0,1,1,0,2,2, 0,2,1,1,2,0) * id;
}
// transform.rs:16-107
void make_matrix(const rs_transform& t, M4 m) {
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) m[i][j] = (i == j) ? 1.0 : 0.0;
    switch (t.kind) {
    case RS_TF_TRANSLATE: m[0][3] = t.v[0]; m[1][3] = t.v[1]; m[2][3] = t.v[2]; break;
    case RS_TF_ROTATE_X: { const double s = std::sin(t.v[0]), c = std::cos(t.v[0]);
        m[1][1] = c; m[1][2] = s; m[2][1] = -s; m[2][2] = c; break; }
    case RS_TF_ROTATE_Y: { const double s = std::sin(t.v[0]), c = std::cos(t.v[0]);
        m[0][0] = c; m[0][2] = s; m[2][0] = -s; m[2][2] = c; break; }
    case RS_TF_ROTATE_Z: { const double s = std::sin(t.v[0]), c = std::cos(t.v[0]);
        m[0][0] = c; m[0][1] = s; m[1][0] = -s; m[1][1] = c; break; }
    case RS_TF_SCALE: m[0][0] = t.v[0]; m[1][1] = t.v[1]; m[2][2] = t.v[2]; m[3][3] = 1.0; break;
    default: throw Error(RS_E_INVALID, "unknown transform kind");
    }
}
void apply34(const M4 m, const double p[3], double w, double out[3]) {
    double r[3];
    for (int i = 0; i < 3; ++i) r[i] = m[i][0] * p[0] + m[i][1] * p[1] + m[i][2] * p[2] + m[i][3] * w;
    out[0] = r[0]; out[1] = r[1]; out[2] = r[2];
}

}  // namespace

// The committed scene in device layout, built once on the host: the DScene template (scalars set,
// pointers null) plus one byte blob per device array and the DScene field that points to it.
struct Blob {
    size_t field_off;            // offset of the pointer field in DScene
    std::vector<char> bytes;
};
struct HostScene {
    DScene ds{};
    std::vector<Blob> blobs;
};

// One frame in flight on a replica: its streams and the render workspace it owns (grown on demand).
// Frames are dealt to a replica's slots round robin; a frame waits only for the previous frame of
// ITS slot (free_ev, recorded after the last kernel that reads the slot's buffers), so the next
// frame's first iterations run while the previous frame's last paths drain.
struct Slot {
    hipStream_t lane[kMaxLanes] = {nullptr};   // lane[0]: the slot's stream; 1..: chunk lanes
    hipEvent_t fork_ev = nullptr, join_ev[kMaxLanes] = {nullptr};
    hipEvent_t free_ev = nullptr, entry_ev = nullptr;
    bool free_rec = false;
    double* d_rad = nullptr; size_t rad_cap = 0;
    double* d_acc = nullptr; size_t acc_cap = 0;
    unsigned long long* d_cnt = nullptr;     // megakernel segment counters (512)
    uint8_t* d_mask = nullptr; size_t mask_cap = 0;   // replicas > 0: the caller's mask copied over
    float* d_out = nullptr; size_t out_cap = 0;       // replicas > 0 / rs_render: the frame on this device
    // wavefront path state (capacity wf_cap paths per set) per lane + queue counters
    void* d_wf = nullptr; size_t wf_cap = 0; uint32_t wf_lanes = 0; size_t wf_bytes = 0;
    QEnt** d_qptrs[kMaxLanes] = {nullptr};        // per lane: device array of the per-class queues
    QEnt* qptr[kMaxLanes][kWfsClasses] = {{nullptr}};
    WfState lane_ws[kMaxLanes]{};
    uint32_t* d_counts = nullptr; size_t counts_cap = 0;
    size_t counts_clean = 0;  // leading entries of d_counts known to be zero (reset by the last frame's accumulate)
    hipStream_t acc_stream = nullptr;         // streaming wavefront: the batches' accumulates
    std::vector<hipEvent_t> bev;              // per batch: its paths done, its accumulate done
    // the carried-path counts of the slot's last streaming frame (per lane and iteration), copied into pinned host
    // memory at its end: they size the carried-extend grids of later frames of the same shape (Replica::hist)
    uint32_t* h_hist = nullptr; size_t hist_cap = 0, hist_words = 0; uint64_t hist_sig = 0;
    hipEvent_t hist_ev = nullptr; bool hist_pending = false;

    // wait until nothing in flight uses this slot's buffers
    void quiesce() {
        for (uint32_t l = 0; l < kMaxLanes; ++l)
            if (lane[l]) HIP_OK(hipStreamSynchronize(lane[l]));
        if (acc_stream) HIP_OK(hipStreamSynchronize(acc_stream));
        if (free_rec) HIP_OK(hipEventSynchronize(free_ev));
    }
    void release() {
        for (uint32_t l = 0; l < kMaxLanes; ++l)
            if (lane[l]) (void)hipStreamSynchronize(lane[l]);
        if (acc_stream) (void)hipStreamSynchronize(acc_stream);
        if (free_rec) (void)hipEventSynchronize(free_ev);
        for (void* p : {(void*)d_rad, (void*)d_acc, (void*)d_cnt, (void*)d_mask, (void*)d_out, d_wf, (void*)d_counts})
            if (p) (void)hipFree(p);
        for (uint32_t l = 0; l < kMaxLanes; ++l) {
            if (lane[l]) (void)hipStreamDestroy(lane[l]);
            if (join_ev[l]) (void)hipEventDestroy(join_ev[l]);
        }
        for (hipEvent_t e : {fork_ev, free_ev, entry_ev})
            if (e) (void)hipEventDestroy(e);
        for (hipEvent_t e : bev) (void)hipEventDestroy(e);
        if (acc_stream) (void)hipStreamDestroy(acc_stream);
        if (hist_ev) (void)hipEventDestroy(hist_ev);
        if (h_hist) (void)hipHostFree(h_hist);
    }
};

// One device the scene is committed to: its copy of the scene arrays and its frame slots. A device
// may appear more than once in rs_scene_commit_devices (virtual devices, e.g. for tests): every
// replica owns its own streams and buffers.
struct Replica {
    int device = 0;
    hipStream_t stream = nullptr;           // the replica's own stream (multi-device renders, rs_render)
    DScene ds{};
    std::vector<void*> dev;                 // scene allocations
    Slot slots[kMaxSlots];
    uint32_t next_slot = 0;
    int n_cu = 0, ext_bpc = 0, shade_bpc = 0;
    uint64_t mem_total = 0;                 // device memory (bytes): caps the streaming pool (pool_limit)
    int32_t* d_ovf = nullptr; size_t ovf_cap = 0;   // traversal-stack overflow (entries beyond the LDS part)
    DScene* d_ds = nullptr;                 // ds in device memory (what the kernels read)
    DScene uploaded{};                      // the copy last written to d_ds
    std::vector<uint32_t> hist;             // the latest completed streaming frame's carried counts (Slot::h_hist)
    uint64_t hist_sig = 0;                  // and its schedule's signature
    std::vector<hipStream_t> pad_streams;   // dev A/B only (RS_PAD_STREAMS)

    // wait until no frame of this replica is in flight (before a shared buffer is replaced)
    void quiesce() {
        for (Slot& sl : slots) sl.quiesce();
        if (stream) HIP_OK(hipStreamSynchronize(stream));
    }
    // the scene for a launch, with d_ds brought up to date first (it changes only when the
    // stack-overflow array is reallocated)
    SceneRef ref() {
        if (std::memcmp(&uploaded, &ds, sizeof(DScene)) != 0) {
            quiesce();
            HIP_OK(hipMemcpy(d_ds, &ds, sizeof(DScene), hipMemcpyHostToDevice));
            uploaded = ds;
        }
        return SceneRef{&ds, d_ds};
    }

    ~Replica() {
        int prev = -1;
        const bool switched = hipGetDevice(&prev) == hipSuccess && prev != device && hipSetDevice(device) == hipSuccess;
        for (Slot& sl : slots) sl.release();  // an asynchronous frame may still read the scene
        if (stream) (void)hipStreamSynchronize(stream);
        for (hipStream_t st : pad_streams) (void)hipStreamDestroy(st);
        for (void* p : dev) (void)hipFree(p);
        for (void* p : {(void*)d_ovf, (void*)d_ds})
            if (p) (void)hipFree(p);
        if (stream) (void)hipStreamDestroy(stream);
        if (switched) (void)hipSetDevice(prev);
    }
};

struct rs_scene {
    std::vector<rs_material_desc> mdesc;
    std::vector<HPerlin> perlins;
    std::vector<HImage> images;
    std::vector<HObj> objs;
    std::vector<uint32_t> world, lights;
    float bg_lo[3] = {0.3f, 0.4f, 0.5f}, bg_hi[3] = {0.7f, 0.89f, 1.0f};
    bool committed = false;
    bool spheres_only = false;
    int scene_mode = kSmGeneric;        // rs_internal.h SceneMode
    bool ref_order = false;                 // BVH::hit recursion order needed (non-monotone objects)
    HostScene hs;                           // device layout, built once by commit
    std::vector<std::unique_ptr<Replica>> reps;   // the devices the scene is committed to, in call order
    // workspace (rs_scene_set_workspace): camera samples per rad batch buffer; paths per set of the
    // streaming pool / per chunk of the bounce-synchronous wavefront
    uint64_t max_items_per_batch = 32ull << 20;
    // streaming pool bound (paths per set): a frame injects Q samples per iteration with Q * min(depth, iterations)
    // <= the pool, so a larger pool means fewer, fuller iterations on big depth-50 frames (C3 1920x1080x256:
    // 64 Mi 210.9 ms, 128 Mi 197.1 ms, 256 Mi 190.7 ms; profiles/r5/ab/pool_sizes_r5c.jsonl); each replica caps it
    // by its device memory and, when a slot allocates, by what is free (pool_limit, pool_limit_free)
    uint64_t pool_paths = 256ull << 20;
    uint32_t inject_div = 1;                      // streaming: inject up to 1/inject_div of a lane per iteration
    uint32_t finish_after = 16;                   // streaming: wavefront iterations after the last injection before
                                                  // the finish launch (k_wfs_finish; 0: none; never on nest-2 scenes)
    uint32_t wf_lanes = 2;                        // chunk lanes of the bounce-synchronous wavefront (rs_scene_set_lanes)
    uint32_t stream_lanes = 1;                    // lanes of the streaming wavefront (rs_scene_set_lanes)
    uint32_t frames_in_flight = 3;                // frame slots per replica (rs_scene_set_frames_in_flight; 3: bench frame
                                                  // -0.6 %, its N = 8 row share -3 % against 2, profiles/r5/ab/frames_in_flight_r6*)
    bool ext_split = false;                       // streaming extend in two launches per iteration in every mode (dev A/B)
    bool shade_split = true;                      // spheres mode: lean / heavy material classes in two shading launches
    bool dump_iters = false;                      // dev: per-iteration queue counts to stderr (timed frames)
    uint32_t passes_stream = 0;                   // rs_render_device_passes: 0 where it pays, 1 always, 2 never (dev A/B)
    uint32_t class_mask = (1u << kWfsClasses) - 1;  // shading classes some prim has (empty queues are not launched)
    int tree_depth = 0;                     // levels of the tree in use
    int tree_arity = 0;                     // 4: 4-wide tree, 2: binary tree, 0: empty world
    int stack_need = 0;                     // exact worst-case traversal stack depth of that tree
    size_t n_nodes = 0;
    size_t n_leaf_entries = 0;
    double time0 = 0.0, time1 = 0.0;        // World::new time_limit (world.rs:40-53)

    uint32_t add(HObj o) {
        if (committed) throw Error(RS_E_STATE, "scene already committed");
        objs.push_back(std::move(o));
        return (uint32_t)(objs.size() - 1);
    }
    void check_mat(int32_t m) const {
        if (m != RS_NO_MATERIAL && (m < 0 || (size_t)m >= mdesc.size())) throw Error(RS_E_INVALID, "unknown material id");
    }
    void check_handle(uint32_t h) const {
        if (h >= objs.size()) throw Error(RS_E_INVALID, "unknown object handle");
    }

    // reference bbox of each handle over World::new's time range [time0, time1]
    Box3 bbox(uint32_t h) { return bbox_t(h, time0, time1); }
    Box3 bbox_t(uint32_t h, double time0, double time1) {
        const HObj& o = objs[h];
        Box3 r;
        switch (o.kind) {
        case PK_SPHERE: {
            const double* c = o.p; const double rad = o.p[3]; const double* v = o.p + 5;
            Box3 s, e;
            if (v[0] == 0.0 && v[1] == 0.0 && v[2] == 0.0) {
                for (int i = 0; i < 3; ++i) { s.lo[i] = c[i] - rad; s.hi[i] = c[i] + rad; }
                return s;
            }
            for (int i = 0; i < 3; ++i) {
                double c0 = c[i] + v[i] * time0, c1 = c[i] + v[i] * time1;
                s.lo[i] = c0 - rad; s.hi[i] = c0 + rad; e.lo[i] = c1 - rad; e.hi[i] = c1 + rad;
            }
            return box_union(s, e);
        }
        case PK_RECT: {
            r.lo[o.ax[0]] = o.p[1]; r.lo[o.ax[1]] = o.p[3]; r.lo[o.ax[2]] = o.p[0] - 0.0001;
            r.hi[o.ax[0]] = o.p[2]; r.hi[o.ax[1]] = o.p[4]; r.hi[o.ax[2]] = o.p[0] + 0.0001;
            return r;
        }
        case PK_BOX: {
            const double* mn = o.p; const double* mx = o.p + 3;
            // the six faces in box.rs order; union in list order (list.rs:68-81)
            struct F { int ax0, ax1, ax2; double k, a0, a1, b0, b1; } f[6] = {
                {0, 1, 2, mn[2], mn[0], mx[0], mn[1], mx[1]}, {0, 1, 2, mx[2], mn[0], mx[0], mn[1], mx[1]},
                {1, 2, 0, mn[0], mn[1], mx[1], mn[2], mx[2]}, {1, 2, 0, mx[0], mn[1], mx[1], mn[2], mx[2]},
                {0, 2, 1, mn[1], mn[0], mx[0], mn[2], mx[2]}, {0, 2, 1, mx[1], mn[0], mx[0], mn[2], mx[2]}};
            for (int i = 0; i < 6; ++i) {
                Box3 fb;
                fb.lo[f[i].ax0] = f[i].a0; fb.lo[f[i].ax1] = f[i].b0; fb.lo[f[i].ax2] = f[i].k - 0.0001;
                fb.hi[f[i].ax0] = f[i].a1; fb.hi[f[i].ax1] = f[i].b1; fb.hi[f[i].ax2] = f[i].k + 0.0001;
                r = i == 0 ? fb : box_union(r, fb);
            }
            return r;
        }
        case PK_QUADRIC:
            for (int i = 0; i < 3; ++i) { r.lo[i] = -100.0; r.hi[i] = 100.0; }
            return r;
        case PK_TRIANGLE: {
            for (int i = 0; i < 3; ++i) {
                r.lo[i] = std::fmin(std::fmin(o.p[i], o.p[3 + i]), o.p[6 + i]);
                r.hi[i] = std::fmax(std::fmax(o.p[i], o.p[3 + i]), o.p[6 + i]);
            }
            return r;
        }
        case PK_AND: {
            Box3 b1 = bbox_t((uint32_t)o.a, time0, time1), b2 = bbox_t((uint32_t)o.b, time0, time1);
            r.lo[0] = std::fmax(b1.lo[0], b2.lo[0]);
            r.lo[1] = std::fmax(b1.lo[1], b2.lo[1]);
            r.lo[2] = std::fmax(b1.lo[1], b2.lo[2]);  // intersection.rs:110 uses b1.min.y for z
            for (int i = 0; i < 3; ++i) r.hi[i] = std::fmin(b1.hi[i], b2.hi[i]);
            return r;
        }
        case PK_SUB: return bbox_t((uint32_t)o.a, time0, time1);
        case PK_MEDIUM: return bbox_t((uint32_t)o.a, time0, time1);  // constant.rs:93-95
        case PK_XFORM: {
            Box3 b = bbox_t((uint32_t)o.a, time0, time1);
            std::vector<std::vector<double>> fwd;
            r = box_empty();
            for (int i = 0; i < 2; ++i) for (int j = 0; j < 2; ++j) for (int k = 0; k < 2; ++k) {
                double p[3] = {std::fma((double)i, b.hi[0], (double)(1 - i) * b.lo[0]),
                               std::fma((double)j, b.hi[1], (double)(1 - j) * b.lo[1]),
                               std::fma((double)k, b.hi[2], (double)(1 - k) * b.lo[2])};
                for (const rs_transform& t : o.tfs) {
                    M4 m;
                    make_matrix(t, m);
                    apply34(m, p, 1.0, p);
                }
                for (int c = 0; c < 3; ++c) { r.lo[c] = std::fmin(r.lo[c], p[c]); r.hi[c] = std::fmax(r.hi[c], p[c]); }
            }
            return r;
        }
        }
        throw Error(RS_E_INVALID, "unknown object kind");
    }

    // true when hit() over [tmin, e) is hit() over [tmin, inf) filtered by t1 < e: then the
    // closest hit does not depend on the order objects are tested in (up to exact ties)
    bool monotone(uint32_t h) const {
        const HObj& o = objs[h];
        if (o.kind == PK_SPHERE || o.kind == PK_RECT || o.kind == PK_TRIANGLE) return true;
        if (o.kind == PK_XFORM) return monotone((uint32_t)o.a);
        return false;  // Box (outside/t2 depend on the far face), Quadric (a < 0 root order), CSG
    }

    int nest_depth(uint32_t h) const {
        const HObj& o = objs[h];
        if (o.kind == PK_AND || o.kind == PK_SUB)
            return 1 + std::max(nest_depth((uint32_t)o.a), nest_depth((uint32_t)o.b));
        if (o.kind == PK_XFORM || o.kind == PK_MEDIUM) return 1 + nest_depth((uint32_t)o.a);
        return 0;
    }
};

namespace {

// ---------------------------------------------------------------- BVH (binned SAH) ----
// host-side node with exact f64 child boxes; converted to the f32 device node at upload
struct HNode {
    double lo[2][3];
    double hi[2][3];
    int32_t child[2];
};
float round_down_f(double x) {
    if (std::isnan(x)) return (float)x;
    float f = (float)x;
    return ((double)f > x) ? std::nextafter(f, -INFINITY) : f;
}
float round_up_f(double x) {
    if (std::isnan(x)) return (float)x;
    float f = (float)x;
    return ((double)f < x) ? std::nextafter(f, INFINITY) : f;
}
DNode to_device(const HNode& h) {
    DNode d;
    std::memset(&d, 0, sizeof(d));
    for (int c = 0; c < 2; ++c)
        for (int k = 0; k < 3; ++k) { d.lo[c][k] = round_down_f(h.lo[c][k]); d.hi[c][k] = round_up_f(h.hi[c][k]); }
    d.child[0] = h.child[0];
    d.child[1] = h.child[1];
    return d;
}

struct BuildItem { Box3 box; double c[3]; int32_t prim; };

// Leaf entries in tree order (DScene::lprim): leaf code ~e names entry e (rs_layout.h).
// With entries = false (scenes without leaf-ordered copies) a leaf code is ~prim.
struct LeafSink {
    bool entries = true;
    std::vector<int32_t> prims;
    template <typename It>
    int32_t add(It first, It last) {
        const size_t n = (size_t)(last - first);
        if (n != 1) throw Error(RS_E_INVALID, "bad leaf size");
        if (!entries) return ~*first;
        if (prims.size() >= (size_t)INT32_MAX - 1) throw Error(RS_E_UNSUPPORTED, "too many objects for the BVH");
        const int32_t e = (int32_t)prims.size();
        prims.push_back(*first);
        return ~e;
    }
};

struct Builder {
    std::vector<HNode> nodes;
    LeafSink* leaves = nullptr;
    int max_leaf = 1;   // objects per leaf
    int sah_depth = 48; // SAH splits above this depth, median splits below (bounds the depth)
    size_t kSweepMax = 1024;  // full-sweep SAH up to this range size, binned above (RS_SAH_SWEEP overrides)
    static constexpr int kBins = 32;
    int max_depth = 0;
    static double area(const Box3& b) {
        double dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
        if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.0;
        if (!std::isfinite(dx) || !std::isfinite(dy) || !std::isfinite(dz)) return 1e300;
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
    // returns the child code of the subtree over items[b, e)
    int32_t build(std::vector<BuildItem>& it, size_t b, size_t e, int depth, Box3& out_box) {
        if (e - b <= (size_t)max_leaf) {
            out_box = it[b].box;
            std::vector<int32_t> ps;
            for (size_t i = b; i < e; ++i) { out_box = box_union(out_box, it[i].box); ps.push_back(it[i].prim); }
            return leaves->add(ps.begin(), ps.end());
        }
        max_depth = std::max(max_depth, depth + 1);
        Box3 cb = box_empty();
        for (size_t i = b; i < e; ++i)
            for (int k = 0; k < 3; ++k) { cb.lo[k] = std::fmin(cb.lo[k], it[i].c[k]); cb.hi[k] = std::fmax(cb.hi[k], it[i].c[k]); }
        size_t mid = b + (e - b) / 2;
        int axis = 0;
        double ext = -1;
        for (int k = 0; k < 3; ++k) if (cb.hi[k] - cb.lo[k] > ext) { ext = cb.hi[k] - cb.lo[k]; axis = k; }
        bool done = false;
        if (depth < sah_depth && e - b > 2 && ext > 0) {  // SAH above sah_depth, median below: depth <= sah_depth + log2(n)
            double best_cost = INFINITY; int best_axis = -1; size_t best_split = 0;
            if (e - b <= kSweepMax) {
                // small ranges: SAH over a full sweep of the centroid-sorted range on each axis
                std::vector<double> right_area(e - b);
                for (int k = 0; k < 3; ++k) {
                    if (!(cb.hi[k] - cb.lo[k] > 0)) continue;
                    std::stable_sort(it.begin() + b, it.begin() + e, [k](const BuildItem& x, const BuildItem& y) { return x.c[k] < y.c[k]; });
                    Box3 acc = box_empty();
                    for (size_t i = e; i-- > b + 1;) { acc = box_union(acc, it[i].box); right_area[i - b] = area(acc); }
                    acc = box_empty();
                    for (size_t i = b; i + 1 < e; ++i) {
                        acc = box_union(acc, it[i].box);
                        double cost = area(acc) * (double)(i + 1 - b) + right_area[i + 1 - b] * (double)(e - i - 1);
                        if (cost < best_cost) { best_cost = cost; best_axis = k; best_split = i + 1; }
                    }
                }
            } else {
                // large ranges: binned SAH (kBins centroid bins per axis), then the range is ordered on
                // the chosen axis so the left side is the first best_split - b items
                for (int k = 0; k < 3; ++k) {
                    const double lo = cb.lo[k], span = cb.hi[k] - cb.lo[k];
                    if (!(span > 0) || !std::isfinite(span)) continue;
                    const double scale = (double)kBins / span;
                    Box3 bbox[kBins];
                    size_t bcnt[kBins] = {0};
                    for (int q = 0; q < kBins; ++q) bbox[q] = box_empty();
                    for (size_t i = b; i < e; ++i) {
                        const int q = std::min(kBins - 1, std::max(0, (int)((it[i].c[k] - lo) * scale)));
                        bbox[q] = box_union(bbox[q], it[i].box);
                        ++bcnt[q];
                    }
                    double rarea[kBins];
                    size_t rcnt[kBins];
                    Box3 acc = box_empty();
                    size_t n = 0;
                    for (int q = kBins - 1; q >= 1; --q) { acc = box_union(acc, bbox[q]); n += bcnt[q]; rarea[q] = area(acc); rcnt[q] = n; }
                    acc = box_empty();
                    n = 0;
                    for (int q = 0; q + 1 < kBins; ++q) {
                        acc = box_union(acc, bbox[q]);
                        n += bcnt[q];
                        if (n == 0 || rcnt[q + 1] == 0) continue;
                        const double cost = area(acc) * (double)n + rarea[q + 1] * (double)rcnt[q + 1];
                        if (cost < best_cost) { best_cost = cost; best_axis = k; best_split = b + n; }
                    }
                }
            }
            if (best_axis >= 0) {
                std::stable_sort(it.begin() + b, it.begin() + e,
                                 [best_axis](const BuildItem& x, const BuildItem& y) { return x.c[best_axis] < y.c[best_axis]; });
                mid = best_split;
                done = true;
            }
        }
        if (!done) {
            std::stable_sort(it.begin() + b, it.begin() + e, [axis](const BuildItem& x, const BuildItem& y) { return x.c[axis] < y.c[axis]; });
            mid = b + (e - b) / 2;
        }
        const int32_t idx = (int32_t)nodes.size();
        nodes.emplace_back();
        Box3 lb, rb;
        const int32_t l = build(it, b, mid, depth + 1, lb);
        const int32_t r = build(it, mid, e, depth + 1, rb);
        HNode& n = nodes[idx];
        std::memset(&n, 0, sizeof(n));
        for (int k = 0; k < 3; ++k) { n.lo[0][k] = lb.lo[k]; n.hi[0][k] = lb.hi[k]; n.lo[1][k] = rb.lo[k]; n.hi[1][k] = rb.hi[k]; }
        n.child[0] = l; n.child[1] = r;
        out_box = box_union(lb, rb);
        return idx;
    }
};

// BVH::new_internal (bvh.rs:58-113) with find_best_axis (bvh.rs:116-169) instead of the random
// axis and one object per leaf: the tree the CPU oracle builds, so reference-order traversal
// visits objects in the same sequence as the oracle's recursion.
struct RefItem { Box3 box; double key_lo[3]; int32_t prim; };
int32_t build_ref(std::vector<HNode>& nodes, LeafSink& leaves, std::vector<RefItem>& it, size_t b, size_t e, int depth,
                  int& max_depth, Box3& out) {
    if (e - b == 1) { out = it[b].box; return leaves.add(&it[b].prim, &it[b].prim + 1); }
    max_depth = std::max(max_depth, depth + 1);
    Box3 u = it[b].box;
    for (size_t i = b + 1; i < e; ++i) u = box_union(u, it[i].box);
    const double sx = u.hi[0] - u.lo[0], sy = u.hi[1] - u.lo[1], sz = u.hi[2] - u.lo[2];
    int axis = 0;
    if (sx > sy && sx > sz) axis = 0;
    else if (sy > sx && sy > sz) axis = 1;
    else if (sz > sx && sz > sy) axis = 2;
    std::stable_sort(it.begin() + b, it.begin() + e, [axis](const RefItem& p, const RefItem& q) { return p.key_lo[axis] < q.key_lo[axis]; });
    const size_t mid = b + (e - b) / 2;
    const int32_t idx = (int32_t)nodes.size();
    nodes.emplace_back();
    Box3 lb, rb;
    const int32_t l = build_ref(nodes, leaves, it, b, mid, depth + 1, max_depth, lb);
    const int32_t r = build_ref(nodes, leaves, it, mid, e, depth + 1, max_depth, rb);
    HNode& n = nodes[idx];
    std::memset(&n, 0, sizeof(n));
    for (int k = 0; k < 3; ++k) { n.lo[0][k] = lb.lo[k]; n.hi[0][k] = lb.hi[k]; n.lo[1][k] = rb.lo[k]; n.hi[1][k] = rb.hi[k]; }
    n.child[0] = l; n.child[1] = r;
    out = box_union(lb, rb);
    return idx;
}

// Collapse the binary tree into a 4-wide one: repeatedly open the inner child with the largest
// box surface until four slots are filled.
template <int W> struct HNodeW { double lo[W][3], hi[W][3]; int32_t child[W]; };
using HNode4 = HNodeW<4>;
// Near-first trees: a node's slots are its binary subtree's top, the largest-area inner slot opened
// into its two children until W slots are filled (or only leaves remain). (An 8-wide tree for the
// spheres mode measured slower: profiles/r4/ab/bvh8.)
template <int W>
int32_t collapseW(const std::vector<HNode>& bn, int32_t code, std::vector<HNodeW<W>>& out, int depth, int& max_depth) {
    if (code < 0) return code;
    max_depth = std::max(max_depth, depth + 1);
    struct Slot { double lo[3], hi[3]; int32_t c; };
    std::vector<Slot> slots;
    const HNode& n = bn[code];
    for (int k = 0; k < 2; ++k) {
        Slot sl; sl.c = n.child[k];
        for (int a = 0; a < 3; ++a) { sl.lo[a] = n.lo[k][a]; sl.hi[a] = n.hi[k][a]; }
        if (sl.c != INT32_MIN) slots.push_back(sl);
    }
    while (slots.size() < (size_t)W) {
        int best = -1; double best_area = -1;
        for (size_t i = 0; i < slots.size(); ++i) {
            if (slots[i].c < 0) continue;
            const double dx = slots[i].hi[0] - slots[i].lo[0], dy = slots[i].hi[1] - slots[i].lo[1], dz = slots[i].hi[2] - slots[i].lo[2];
            const double ar = dx * dy + dy * dz + dz * dx;
            if (ar > best_area) { best_area = ar; best = (int)i; }
        }
        if (best < 0) break;
        const HNode& m = bn[slots[best].c];
        Slot a, b;
        a.c = m.child[0]; b.c = m.child[1];
        for (int q = 0; q < 3; ++q) { a.lo[q] = m.lo[0][q]; a.hi[q] = m.hi[0][q]; b.lo[q] = m.lo[1][q]; b.hi[q] = m.hi[1][q]; }
        slots.erase(slots.begin() + best);
        slots.push_back(a);
        if (b.c != INT32_MIN) slots.push_back(b);
    }
    const int32_t idx = (int32_t)out.size();
    out.emplace_back();
    int32_t kids[W];
    for (int k = 0; k < W; ++k) kids[k] = (size_t)k < slots.size() ? collapseW<W>(bn, slots[k].c, out, depth + 1, max_depth) : INT32_MIN;
    HNodeW<W>& o = out[idx];
    for (int k = 0; k < W; ++k) {
        o.child[k] = kids[k];
        for (int q = 0; q < 3; ++q) {
            o.lo[k][q] = (size_t)k < slots.size() ? slots[k].lo[q] : INFINITY;
            o.hi[k][q] = (size_t)k < slots.size() ? slots[k].hi[q] : -INFINITY;
        }
    }
    return idx;
}
// Reference-order scenes: collapse the reference's binary tree into a 4-wide one whose slots keep the
// recursion's left-to-right order (an inner slot is replaced IN PLACE by its two children), so a walk
// of the slots in order, each child's box tested when it is reached, visits the objects in
// BVH::hit's sequence with the same ranges (bvh.rs:173-192): a skipped intermediate box contains its
// children's (f32 boxes rounded outward, monotone plane tests), so when it would have failed at range
// r its first child fails at r too, nothing inside it is visited, the range stays r and its second
// child fails as well -- whether or not ranges only shrink (Difference back faces).
int32_t collapse4_inorder(const std::vector<HNode>& bn, int32_t code, std::vector<HNode4>& out, int depth,
                          int& max_depth) {
    if (code < 0) return code;
    max_depth = std::max(max_depth, depth + 1);
    struct Slot { double lo[3], hi[3]; int32_t c; };
    std::vector<Slot> slots;
    auto children = [&](int32_t node, std::vector<Slot>& to, size_t at) {
        const HNode& n = bn[node];
        size_t pos = at;
        for (int k = 0; k < 2; ++k) {
            if (n.child[k] == INT32_MIN) continue;
            Slot sl; sl.c = n.child[k];
            for (int a = 0; a < 3; ++a) { sl.lo[a] = n.lo[k][a]; sl.hi[a] = n.hi[k][a]; }
            to.insert(to.begin() + pos++, sl);
        }
    };
    children(code, slots, 0);
    while (slots.size() < 4) {
        int best = -1; double best_area = -1;
        for (size_t i = 0; i < slots.size(); ++i) {
            if (slots[i].c < 0) continue;
            const double dx = slots[i].hi[0] - slots[i].lo[0], dy = slots[i].hi[1] - slots[i].lo[1], dz = slots[i].hi[2] - slots[i].lo[2];
            const double ar = dx * dy + dy * dz + dz * dx;
            if (ar > best_area) { best_area = ar; best = (int)i; }
        }
        if (best < 0) break;
        const int32_t c = slots[best].c;
        if ((int)slots.size() - 1 + (bn[c].child[0] != INT32_MIN) + (bn[c].child[1] != INT32_MIN) > 4) break;
        slots.erase(slots.begin() + best);
        children(c, slots, (size_t)best);
    }
    const int32_t idx = (int32_t)out.size();
    out.emplace_back();
    int32_t kids[4];
    for (int k = 0; k < 4; ++k) kids[k] = (size_t)k < slots.size() ? collapse4_inorder(bn, slots[k].c, out, depth + 1, max_depth) : INT32_MIN;
    HNode4& o = out[idx];
    for (int k = 0; k < 4; ++k) {
        o.child[k] = kids[k];
        for (int q = 0; q < 3; ++q) {
            o.lo[k][q] = (size_t)k < slots.size() ? slots[k].lo[q] : INFINITY;
            o.hi[k][q] = (size_t)k < slots.size() ? slots[k].hi[q] : -INFINITY;
        }
    }
    return idx;
}
// Exact worst-case stack depth of traverse() (rs_kernels.hip) over a tree: the most entries any
// root-to-node path can leave on the stack.
//  4-wide near-first: a node pushes (inner children hit) - 1 <= (inner children) - 1 entries;
template <int W>
int stack_needW(const std::vector<HNodeW<W>>& n4, int32_t code) {
    if (code < 0) return 0;
    int inner = 0, deepest = 0;
    for (int k = 0; k < W; ++k) {
        const int32_t c = n4[code].child[k];
        if (c >= 0) { ++inner; deepest = std::max(deepest, stack_needW<W>(n4, c)); }
    }
    return std::max(inner - 1, 0) + deepest;
}
int stack_need4(const std::vector<HNode4>& n4, int32_t code) { return stack_needW<4>(n4, code); }
//  4-wide reference order: the node (with its next slot) when an inner child before slot 3 is entered;
int stack_need4_ref(const std::vector<HNode4>& n4, int32_t code) {
    if (code < 0) return 0;
    int need = 0;
    for (int k = 0; k < 4; ++k) {
        const int32_t c = n4[code].child[k];
        if (c >= 0) need = std::max(need, (k < 3 ? 1 : 0) + stack_need4_ref(n4, c));
    }
    return need;
}
//  binary near-first: one entry (the farther child) when both children are inner nodes;
int stack_need2(const std::vector<HNode>& bn, int32_t code) {
    if (code < 0) return 0;
    const int32_t c0 = bn[code].child[0], c1 = bn[code].child[1];
    const int a = stack_need2(bn, c0), b = stack_need2(bn, c1);
    return (c0 >= 0 && c1 >= 0 ? 1 : 0) + std::max(a, b);
}
//  binary reference order: the node itself while its left (inner) subtree is searched.
int stack_need_ref(const std::vector<HNode>& bn, int32_t code) {
    if (code < 0) return 0;
    const int32_t c0 = bn[code].child[0], c1 = bn[code].child[1];
    return std::max(c0 >= 0 ? 1 + stack_need_ref(bn, c0) : 0, c1 >= 0 ? stack_need_ref(bn, c1) : 0);
}

DNode4 to_device4(const HNode4& h) {
    DNode4 d;
    std::memset(&d, 0, sizeof(d));
    for (int k = 0; k < 4; ++k) {
        d.lo_x[k] = round_down_f(h.lo[k][0]); d.lo_y[k] = round_down_f(h.lo[k][1]); d.lo_z[k] = round_down_f(h.lo[k][2]);
        d.hi_x[k] = round_up_f(h.hi[k][0]); d.hi_y[k] = round_up_f(h.hi[k][1]); d.hi_z[k] = round_up_f(h.hi[k][2]);
        d.child[k] = h.child[k];
    }
    return d;
}

template <typename T>
void stage(rs_scene* s, const T*& field, const std::vector<T>& v) {
    field = nullptr;  // set per replica (upload_replica); an empty array stays null
    if (v.empty()) return;
    Blob b;
    b.field_off = (size_t)((const char*)&field - (const char*)&s->hs.ds);
    b.bytes.assign((const char*)v.data(), (const char*)v.data() + v.size() * sizeof(T));
    s->hs.blobs.push_back(std::move(b));
}

// The LDS image of a nest-mode scene (DScene::limg): the staged tables a traversal reads, each at a
// 16-byte aligned offset of one blob, when they fit kLimgMax (quadric.sdl: ~3 KB). The tables stay
// in their own arrays too (the shading kernels and the other paths read those).
void build_limg(rs_scene* s) {
    DScene& d = s->hs.ds;
    d.limg = nullptr;
    d.limg_bytes = 0;
    std::memset(d.limg_off, 0, sizeof(d.limg_off));
    if (s->scene_mode != kSmNest0 && s->scene_mode != kSmNest2) return;
    // the image's kernels walk the in-order 4-wide tree with their leaf list in the LDS stack's top
    // kLeafBatch entries (rs_kernels.hip traverse_deferred)
    if (d.root4 < 0 || !d.ref_order || s->stack_need + (int)kLeafBatch > stack_lds(s->scene_mode)) return;
    const uint32_t cap = kLimgMax;
#ifdef RS_DEV_KNOBS
    if (std::getenv("RS_NO_LIMG")) return;  // the tables in global memory, for comparison
#endif
    const void* const* fields[LT_COUNT] = {
        (const void* const*)&d.nodes4, (const void* const*)&d.pbox, (const void* const*)&d.pclass,
        (const void* const*)&d.prims, (const void* const*)&d.spheres, (const void* const*)&d.rects,
        (const void* const*)&d.boxes, (const void* const*)&d.quadrics, (const void* const*)&d.csgs,
        (const void* const*)&d.xforms, (const void* const*)&d.tf_fwd, (const void* const*)&d.tf_inv};
    std::vector<char> img;
    for (int t = 0; t < LT_COUNT; ++t) {
        const size_t fo = (size_t)((const char*)fields[t] - (const char*)&d);
        img.resize((img.size() + 15) & ~(size_t)15);
        d.limg_off[t] = (uint32_t)img.size();
        for (const Blob& b : s->hs.blobs)
            if (b.field_off == fo) img.insert(img.end(), b.bytes.begin(), b.bytes.end());
        if (img.size() > cap) return;
    }
    img.resize((img.size() + 15) & ~(size_t)15);
    if (img.size() > cap) return;
    d.limg_bytes = (uint32_t)img.size();
    Blob b;
    b.field_off = (size_t)((const char*)&d.limg - (const char*)&d);
    b.bytes = std::move(img);
    s->hs.blobs.push_back(std::move(b));
}

// copy the staged scene to `device` as a new replica
void upload_replica(rs_scene* s, int device) {
    std::unique_ptr<Replica> R(new Replica());
    R->device = device;
    HIP_OK(hipSetDevice(device));
    R->ds = s->hs.ds;
    for (const Blob& b : s->hs.blobs) {
        void* p = nullptr;
        HIP_OK(hipMalloc(&p, b.bytes.size()));
        R->dev.push_back(p);
        HIP_OK(hipMemcpy(p, b.bytes.data(), b.bytes.size(), hipMemcpyHostToDevice));
        std::memcpy((char*)&R->ds + b.field_off, &p, sizeof(void*));
    }
    HIP_OK(hipMalloc((void**)&R->d_ds, sizeof(DScene)));
    std::memset(&R->uploaded, 0xff, sizeof(DScene));  // forces the first upload
    HIP_OK(hipStreamCreateWithFlags(&R->stream, hipStreamNonBlocking));
#ifdef RS_DEV_KNOBS  // dev A/B: idle streams created before the slots' streams (they shift HIP's stream -> hardware queue map)
    if (const char* e = std::getenv("RS_PAD_STREAMS"))
        for (int k = std::atoi(e); k > 0; --k) {
            hipStream_t st;
            HIP_OK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
            R->pad_streams.push_back(st);
        }
#endif
    hipDeviceProp_t prop;
    HIP_OK(hipGetDeviceProperties(&prop, device));
    R->n_cu = prop.multiProcessorCount;
    R->mem_total = (uint64_t)prop.totalGlobalMem;
    HIP_OK(wf_occupancy(s->scene_mode, &R->ext_bpc, &R->shade_bpc));
    s->reps.push_back(std::move(R));
}

// Build the device layout of the scene on the host (BVH, flattened objects, materials, textures).
void build(rs_scene* s) {
    if (s->committed) throw Error(RS_E_STATE, "scene already committed");
    s->hs = HostScene();
    for (uint32_t h : s->world) if (s->nest_depth(h) > RS_MAX_NEST) throw Error(RS_E_UNSUPPORTED, "object nesting deeper than the GPU path supports");
    for (uint32_t h : s->lights) if (s->nest_depth(h) > RS_MAX_NEST) throw Error(RS_E_UNSUPPORTED, "light nesting deeper than the GPU path supports");

    // materials (+ the world default material, world.rs:51)
    std::vector<DMaterial> mats;
    for (const rs_material_desc& d : s->mdesc) {
        DMaterial m;
        std::memset(&m, 0, sizeof(m));
        m.kind = d.kind; m.tex_kind = d.texture.kind; m.tex_data = d.texture.data; m.glass = d.glass;
        m.k_specular = d.k_specular;
        m.mix_a = d.mix_a; m.mix_b = d.mix_b;
        for (int i = 0; i < 4; ++i) { m.even[i] = d.texture.even[i]; m.odd[i] = d.texture.odd[i]; }
        m.tex_scale = d.texture.scale;
        m.enter_refractive = 1.0 / d.refractive;   // dielectric.rs:38-46
        m.outer_refractive = d.refractive;
        m.exponent = d.exponent; m.multiplier = d.multiplier; m.mix_p = d.mix_p;
        // settings(): MixedMaterial forwards material_1's (mixed_material.rs:56-58)
        const rs_material_desc* e = &d;
        for (int k = 0; k < 64 && e->kind == RS_MAT_MIXED; ++k) e = &s->mdesc[e->mix_a];
        m.phong_factor = e->phong_factor; m.phong_exponent = e->phong_exponent;
        mats.push_back(m);
    }
    DMaterial dm;
    std::memset(&dm, 0, sizeof(dm));
    dm.kind = RS_MAT_LAMBERTIAN; dm.tex_kind = RS_TEX_SOLID;
    for (int i = 0; i < 4; ++i) dm.even[i] = 1.0f;
    dm.enter_refractive = dm.outer_refractive = 1.0; dm.multiplier = 1.0; dm.phong_exponent = 1;
    const int32_t default_mat = (int32_t)mats.size();
    mats.push_back(dm);

    // lights are needed when any pdf material can be hit (list.rs:51 would panic on % 0)
    bool needs_lights = false;
    for (const rs_material_desc& d : s->mdesc)
        if (d.kind == RS_MAT_LAMBERTIAN || d.kind == RS_MAT_DIFFUSE_METAL || d.kind == RS_MAT_MIXED ||
            d.kind == RS_MAT_ISOTROPIC || d.kind == RS_MAT_BLINN_PHONG)
            needs_lights = true;
    for (uint32_t h : s->world) {
        const HObj& o = s->objs[h];
        if (o.mat == RS_NO_MATERIAL && o.kind <= PK_TRIANGLE) needs_lights = true;
    }
    if (needs_lights && s->lights.empty())
        throw Error(RS_E_NO_LIGHTS, "scene has pdf materials but an empty lights list (reference: % 0 panic, list.rs:51)");

    // flatten every handle
    std::vector<DPrim> prims(s->objs.size());
    std::vector<DSphere> spheres; std::vector<DRect> rects; std::vector<DBox> boxes; std::vector<DQuadric> quads;
    std::vector<DTri> tris; std::vector<DCsg> csgs; std::vector<DXform> xforms; std::vector<DMat34> tf_f, tf_i;
    std::vector<DMedium> media;
    for (size_t h = 0; h < s->objs.size(); ++h) {
        const HObj& o = s->objs[h];
        DPrim& P = prims[h];
        P.kind = o.kind; P.mat = o.mat; P.aux = 0;
        switch (o.kind) {
        case PK_SPHERE: {
            DSphere x; for (int i = 0; i < 3; ++i) { x.c[i] = o.p[i]; x.v[i] = o.p[5 + i]; }
            x.r = o.p[3]; x.r2 = o.p[4];
            P.idx = (int32_t)spheres.size(); spheres.push_back(x); break;
        }
        case PK_RECT: {
            DRect x; x.ax0 = o.ax[0]; x.ax1 = o.ax[1]; x.ax2 = o.ax[2]; x.pad = 0;
            x.k = o.p[0]; x.a0 = o.p[1]; x.a1 = o.p[2]; x.b0 = o.p[3]; x.b1 = o.p[4];
            P.idx = (int32_t)rects.size(); rects.push_back(x); break;
        }
        case PK_BOX: {
            DBox x; for (int i = 0; i < 3; ++i) { x.mn[i] = o.p[i]; x.mx[i] = o.p[3 + i]; }
            P.idx = (int32_t)boxes.size(); boxes.push_back(x); break;
        }
        case PK_QUADRIC: {
            DQuadric x; for (int i = 0; i < 10; ++i) x.q[i] = o.p[i];
            P.idx = (int32_t)quads.size(); quads.push_back(x); break;
        }
        case PK_TRIANGLE: {
            DTri x;
            const double* p0 = o.p; const double* p1 = o.p + 3; const double* p2 = o.p + 6;
            for (int i = 0; i < 3; ++i) x.p0[i] = p0[i];
            x.a = p0[0] - p1[0]; x.b = p0[1] - p1[1]; x.c = p0[2] - p1[2];   // triangle_mesh.rs:42-58
            x.d = p0[0] - p2[0]; x.e = p0[1] - p2[1]; x.f = p0[2] - p2[2];
            for (int i = 0; i < 3; ++i) { x.n0[i] = o.p[9 + i]; x.n1[i] = o.p[12 + i]; x.n2[i] = o.p[15 + i]; }
            P.idx = (int32_t)tris.size(); tris.push_back(x); break;
        }
        case PK_AND: case PK_SUB: {
            DCsg x; x.a = o.a; x.b = o.b;
            P.idx = (int32_t)csgs.size(); csgs.push_back(x); break;
        }
        case PK_XFORM: {
            DXform x; x.child = o.a; x.first = (int32_t)tf_f.size();
            for (const rs_transform& t : o.tfs) {
                M4 m, mi;
                make_matrix(t, m);
                inv4(m, mi);
                DMat34 a, b;
                for (int i = 0; i < 3; ++i) for (int j = 0; j < 4; ++j) { a.m[i][j] = m[i][j]; b.m[i][j] = mi[i][j]; }
                tf_f.push_back(a); tf_i.push_back(b);
            }
            P.aux = (int32_t)o.tfs.size();
            P.idx = (int32_t)xforms.size(); xforms.push_back(x); break;
        }
        case PK_MEDIUM: {
            DMedium x; x.boundary = o.a; x.mat = o.mat; x.neg_inv_density = o.p[0];
            P.idx = (int32_t)media.size(); media.push_back(x); break;
        }
        default: throw Error(RS_E_INVALID, "unknown object kind");
        }
    }

    // BVH over the world list (duplicates in the list are kept as separate leaves, like the reference)
    std::vector<BuildItem> items;
    s->spheres_only = true;
    for (uint32_t h : s->world) {
        BuildItem bi;
        bi.box = s->bbox(h);
        for (int k = 0; k < 3; ++k) {
            double lo = bi.box.lo[k], hi = bi.box.hi[k];
            bi.c[k] = (std::isfinite(lo) && std::isfinite(hi)) ? 0.5 * (lo + hi) : 0.0;
        }
        bi.prim = (int32_t)h;
        items.push_back(bi);
        if (s->objs[h].kind != PK_SPHERE) s->spheres_only = false;
    }
    for (uint32_t h : s->lights) if (s->objs[h].kind != PK_SPHERE) s->spheres_only = false;
    bool flat = true;  // only leaf kinds without nesting or order dependence
    auto leaf_kind = [&](uint32_t h) {
        const int k = s->objs[h].kind;
        return k == PK_SPHERE || k == PK_RECT || k == PK_TRIANGLE;
    };
    for (uint32_t h : s->world) flat = flat && leaf_kind(h);
    for (uint32_t h : s->lights) flat = flat && leaf_kind(h);
    int nest = 0;
    for (uint32_t h : s->world) nest = std::max(nest, s->nest_depth(h));
    for (uint32_t h : s->lights) nest = std::max(nest, s->nest_depth(h));
    // the rich features (ConstantMedium, Isotropic / BlinnPhong, Perlin / Image textures) exist only in
    // the generic mode
    bool rich = false;
    for (const HObj& o : s->objs) rich = rich || o.kind == PK_MEDIUM;
    for (const rs_material_desc& d : s->mdesc)
        rich = rich || d.texture.kind == RS_TEX_PERLIN || d.texture.kind == RS_TEX_IMAGE || d.kind == RS_MAT_ISOTROPIC ||
               d.kind == RS_MAT_BLINN_PHONG;
    if (rich) s->spheres_only = false;
    s->scene_mode = rich ? kSmGeneric : s->spheres_only ? kSmSpheres : flat ? kSmFlat : nest == 0 ? kSmNest0 : nest <= 2 ? kSmNest2 : kSmGeneric;
    bool all_monotone = true;
    for (uint32_t h : s->world) all_monotone = all_monotone && s->monotone(h);
    s->ref_order = !all_monotone;
    Builder B;
    LeafSink leaves;
    leaves.entries = s->scene_mode == kSmFlat;
    B.leaves = &leaves;
    // one object per leaf (measured on the C5 mesh: 2, 4 and 8 objects per leaf were 15 %, 45 % and
    // 100 % slower -- a wave serialises its lanes' longer leaf loops)
    B.max_leaf = 1;
#ifdef RS_DEV_KNOBS
    if (const char* ev = std::getenv("RS_SAH_DEPTH")) B.sah_depth = std::max(0, std::atoi(ev));
    if (const char* ev = std::getenv("RS_SAH_SWEEP")) B.kSweepMax = (size_t)std::max(2LL, std::atoll(ev));
#endif
    int32_t root = -1;
    if (!items.empty()) {
        Box3 rb;
        int32_t code;
        if (s->ref_order) {
            std::vector<RefItem> ri;
            for (uint32_t h : s->world) {
                RefItem x;
                x.box = s->bbox(h);
                const Box3 k = s->bbox_t(h, 0.0, 0.0);  // cmp_geometry_by sorts on bbox(0..0).min (bvh.rs:30-43)
                for (int a = 0; a < 3; ++a) x.key_lo[a] = k.lo[a];
                x.prim = (int32_t)h;
                ri.push_back(x);
            }
            code = build_ref(B.nodes, leaves, ri, 0, ri.size(), 0, B.max_depth, rb);
        } else {
            code = B.build(items, 0, items.size(), 0, rb);
        }
        if (code < 0) {  // a single object: wrap it in one node (second slot empty)
            HNode n;
            std::memset(&n, 0, sizeof(n));
            for (int k = 0; k < 3; ++k) { n.lo[0][k] = rb.lo[k]; n.hi[0][k] = rb.hi[k]; n.lo[1][k] = INFINITY; n.hi[1][k] = -INFINITY; }
            n.child[0] = code; n.child[1] = INT32_MIN;
            B.nodes.push_back(n);
            root = 0;
            B.max_depth = 1;
        } else {
            root = code;
        }
    }
    s->tree_depth = B.max_depth;

    std::vector<int32_t> lights(s->lights.begin(), s->lights.end());
    DScene& d = s->hs.ds;
    std::memset(&d, 0, sizeof(d));
    std::vector<DNode> dnodes;
    for (const HNode& h : B.nodes) dnodes.push_back(to_device(h));
    std::vector<DBox64> pboxes(s->objs.size());
    for (size_t h = 0; h < s->objs.size(); ++h) {
        const Box3 b = s->bbox((uint32_t)h);
        for (int k = 0; k < 3; ++k) { pboxes[h].lo[k] = b.lo[k]; pboxes[h].hi[k] = b.hi[k]; }
    }
    // wavefront shading class per prim: the class of every material a record of its hit can carry.
    // A TfFacade passes its child's record (tf_facade.rs:41-55); an Intersection returns either
    // child's record with set_material_if_none (intersection.rs:81-92, hit.rs:69-78); a Difference
    // the plus record as is or with set_material_if_none, or a back-face record carrying the minus
    // object's own material (difference.rs:57-106). When all of them are one class the prim gets it
    // (quadric.sdl's translated quadric-box intersections: Lambertian), else the generic class 4.
    // Light class 6 (emission inside extend) only for leaves and TfFacades of leaves.
    std::vector<uint8_t> pclass(s->objs.size(), 4);
    auto mat_class = [&](int32_t m) -> int {
        const int k = mats[m >= 0 ? m : default_mat].kind;
        return k == RS_MAT_LAMBERTIAN ? 0 : k == RS_MAT_METAL ? 1 : k == RS_MAT_DIFFUSE_METAL ? 2
             : k == RS_MAT_DIELECTRIC ? 3 : k == RS_MAT_DIFFUSE_LIGHT ? 6 : 4;
    };
    // record materials (RS_NO_MATERIAL = None) a hit of prim h can carry; false: unknown / media
    std::function<bool(uint32_t, std::vector<int32_t>&)> rec_mats = [&](uint32_t h, std::vector<int32_t>& out) -> bool {
        const HObj& o = s->objs[h];
        if (o.kind == PK_XFORM) return rec_mats((uint32_t)o.a, out);
        if (o.kind == PK_MEDIUM) return false;
        if (o.kind == PK_AND || o.kind == PK_SUB) {
            std::vector<int32_t> c;
            if (!rec_mats((uint32_t)o.a, c)) return false;
            if (o.kind == PK_AND && !rec_mats((uint32_t)o.b, c)) return false;
            for (int32_t m : c) {
                out.push_back(m != RS_NO_MATERIAL ? m : o.mat);
                if (o.kind == PK_SUB) out.push_back(m);  // the plus record returned as is
            }
            if (o.kind == PK_SUB) {
                const HObj& mo = s->objs[o.b];  // minus->material(): a leaf's own, None for composites
                const bool leaf = mo.kind != PK_AND && mo.kind != PK_SUB && mo.kind != PK_XFORM && mo.kind != PK_MEDIUM;
                const int32_t mm = leaf ? mo.mat : RS_NO_MATERIAL;
                out.push_back(mm != RS_NO_MATERIAL ? mm : o.mat);
            }
            return true;
        }
        out.push_back(o.mat);
        return true;
    };
    std::function<bool(uint32_t)> is_leafish = [&](uint32_t h) -> bool {
        const HObj& o = s->objs[h];
        if (o.kind == PK_XFORM) return is_leafish((uint32_t)o.a);
        return o.kind != PK_AND && o.kind != PK_SUB && o.kind != PK_MEDIUM;
    };
    // Composite prims (CSG, TfFacades of CSG) keep the generic class 4 even when their records are
    // one class: the class queues also sort paths by the object they hit, and a shading wave that
    // mixes CSG hits (finish_hit through the nested-object code) with leaf hits, and the next
    // extend's waves of rays leaving both, run the union of both paths (C4, quadric.sdl at depth
    // 50: 46.1 ms per 512x512x64 frame with CSG in class 4, 56.7 ms with it Lambertian-class).
    auto class_of = [&](uint32_t h) -> int {
        std::vector<int32_t> ms;
        if (!is_leafish(h)) return 4;
        if (!rec_mats(h, ms) || ms.empty()) return 4;
        const int c0 = mat_class(ms[0]);
        for (int32_t m : ms)
            if (mat_class(m) != c0) return 4;
        if (c0 == 6 && !is_leafish(h)) return 4;
        return c0;
    };
    s->class_mask = 0;
    for (size_t h = 0; h < s->objs.size(); ++h) {
        pclass[h] = (uint8_t)class_of((uint32_t)h);
        if (pclass[h] < kWfsClasses) s->class_mask |= 1u << pclass[h];
    }
    d.lamb_only = 1;
    for (size_t h = 0; h < s->objs.size(); ++h) d.lamb_only &= (int32_t)(pclass[h] == 0 || pclass[h] == 6);
    stage(s, d.nodes, dnodes);
    stage(s, d.pbox, pboxes);
    stage(s, d.pclass, pclass);
    d.root4 = -1;
    d.ltop = 0;
    s->tree_arity = root >= 0 ? 2 : 0;
    s->n_nodes = B.nodes.size();
    // the binary tree is walked in reference order by ref_order scenes and, whatever ref_order says,
    // by the nest-0 / nest-2 modes (traverse_body), near-first otherwise: size for the larger need
    if (root >= 0)
        s->stack_need = s->ref_order ? stack_need_ref(B.nodes, root)
                                     : std::max(stack_need_ref(B.nodes, root), stack_need2(B.nodes, root));
    if (!s->ref_order && root >= 0) {
        std::vector<HNode4> n4;
        int depth4 = 0;
        const int32_t r4 = collapseW<4>(B.nodes, root, n4, 0, depth4);
        if (r4 >= 0) {
            // the kernels address nodes with 32-bit byte offsets (rs_kernels.hip gld)
            if (n4.size() * sizeof(DNode4) > 0xFFFFFFFFull) throw Error(RS_E_INVALID, "scene too large: 4-wide tree over 4 GiB");
            s->stack_need = stack_need4(n4, r4);
            int32_t root_id = r4;
            d.ltop = 0;
            // (the flat mode's extend with a 21-node top in LDS measured 1.8 % slower on C5: profiles/r5/configs_r5k.jsonl)
            if (s->scene_mode == kSmSpheres) {
                // the tree's top levels first, breadth-first (nodes 0 .. ltop - 1, which the extend's blocks also hold
                // in LDS: d.ltop), then the other nodes in their depth-first order (a subtree's nodes stay together);
                // the order changes no hit (near-first traversal of the same tree)
                const size_t K = std::min<size_t>(n4.size(), (size_t)kLTop);
                std::vector<int32_t> order, newid(n4.size(), -1);
                order.push_back(r4);
                newid[r4] = 0;
                for (size_t q = 0; q < order.size() && order.size() < K; ++q)
                    for (int k = 0; k < 4 && order.size() < K; ++k) {
                        const int32_t c = n4[order[q]].child[k];
                        if (c >= 0) { newid[c] = (int32_t)order.size(); order.push_back(c); }
                    }
                for (size_t v = 0; v < n4.size(); ++v)
                    if (newid[v] < 0) { newid[v] = (int32_t)order.size(); order.push_back((int32_t)v); }
                std::vector<HNode4> bfs(order.size());
                for (size_t q = 0; q < order.size(); ++q) {
                    bfs[q] = n4[order[q]];
                    for (int k = 0; k < 4; ++k)
                        if (bfs[q].child[k] >= 0) bfs[q].child[k] = newid[bfs[q].child[k]];
                }
                n4.swap(bfs);
                root_id = 0;
                d.ltop = (int32_t)K;
            }
            std::vector<DNode4> dn4;
            for (const HNode4& h : n4) dn4.push_back(to_device4(h));
            stage(s, d.nodes4, dn4);
            d.root4 = root_id;
            s->tree_arity = 4;
            s->tree_depth = depth4;
            s->n_nodes = n4.size();
        }
    }
    // reference-order scenes on the in-order 4-wide tree (collapse4_inorder), nest-0 / nest-2 modes (the
    // generic mode measured 3 % slower on it: X2)
#ifndef RS_GENERIC_4W_MIN
#define RS_GENERIC_4W_MIN 0xFFFFFFFFu
#endif
    const bool inorder4 = s->scene_mode == kSmNest0 || s->scene_mode == kSmNest2 ||
                          (s->scene_mode == kSmGeneric && s->world.size() >= (size_t)RS_GENERIC_4W_MIN);
    if (s->ref_order && inorder4 && root >= 0) {
        std::vector<HNode4> n4;
        int depth4 = 0;
        const int32_t r4 = collapse4_inorder(B.nodes, root, n4, 0, depth4);
        if (r4 >= 0) {
            if (n4.size() * sizeof(DNode4) > 0xFFFFFFFFull) throw Error(RS_E_INVALID, "scene too large: 4-wide tree over 4 GiB");
            std::vector<DNode4> dn4;
            for (const HNode4& h : n4) dn4.push_back(to_device4(h));
            stage(s, d.nodes4, dn4);
            d.root4 = r4;
            s->tree_arity = 4;
            s->tree_depth = depth4;
            s->n_nodes = n4.size();
            s->stack_need = stack_need4_ref(n4, r4);
        }
    }
    d.stack_need = s->stack_need;
    d.moving = 0;
    for (const DSphere& sp : spheres)
        if (sp.v[0] != 0.0 || sp.v[1] != 0.0 || sp.v[2] != 0.0) d.moving = 1;
    d.stk_ovf = nullptr;  // sized per launch grid (ensure_stack_overflow)
    stage(s, d.prims, prims);
    stage(s, d.spheres, spheres);
    // leaf entries in tree order + what each mode's leaf test reads, contiguous per leaf
    stage(s, d.lprim, leaves.prims);
    s->n_leaf_entries = leaves.prims.size();
    if (s->scene_mode == kSmSpheres) {  // prim-indexed sphere copy (leaf codes name prims in this mode)
        std::vector<DSphere> lsph(s->objs.size());
        std::memset(lsph.data(), 0, lsph.size() * sizeof(DSphere));
        for (size_t h = 0; h < s->objs.size(); ++h)
            if (s->objs[h].kind == PK_SPHERE) lsph[h] = spheres[prims[h].idx];
        // the kernels address this array with 32-bit byte offsets (rs_kernels.hip ld_sphere)
        if (lsph.size() * sizeof(DSphere) > 0xFFFFFFFFull) throw Error(RS_E_INVALID, "scene too large: sphere array over 4 GiB");
        if (d.moving) {
            stage(s, d.lsph, lsph);
        } else {  // 32-byte records (DSphereS): the static spheres' leaf data in half the cache lines
            std::vector<DSphereS> lsphs(lsph.size());
            for (size_t h = 0; h < lsph.size(); ++h) {
                for (int k = 0; k < 3; ++k) lsphs[h].c[k] = lsph[h].c[k];
                lsphs[h].r = lsph[h].r;
                if (s->objs[h].kind == PK_SPHERE && lsph[h].r * lsph[h].r != lsph[h].r2)
                    throw Error(RS_E_INVALID, "sphere radius_squared is not radius * radius");
            }
            stage(s, d.lsphs, lsphs);
        }
    }
    if (s->scene_mode == kSmFlat) {
        std::vector<LTri> ltri(leaves.prims.size());
        std::memset(ltri.data(), 0, ltri.size() * sizeof(LTri));
        for (size_t e = 0; e < ltri.size(); ++e) {
            const DPrim& P = prims[leaves.prims[e]];
            ltri[e].kind = (double)P.kind;
            if (P.kind != PK_TRIANGLE) continue;
            const DTri& T = tris[P.idx];
            for (int k = 0; k < 3; ++k) ltri[e].p0[k] = T.p0[k];
            ltri[e].a = T.a; ltri[e].b = T.b; ltri[e].c = T.c; ltri[e].d = T.d; ltri[e].e = T.e; ltri[e].f = T.f;
        }
        // the kernels address this array with 32-bit byte offsets (rs_kernels.hip ld_ltri): ~53.7 M entries
        if (ltri.size() * sizeof(LTri) > 0xFFFFFFFFull) throw Error(RS_E_INVALID, "scene too large: leaf triangle array over 4 GiB");
        stage(s, d.ltri, ltri);
    }
    stage(s, d.rects, rects);
    stage(s, d.boxes, boxes);
    stage(s, d.quadrics, quads);
    stage(s, d.tris, tris);
    stage(s, d.csgs, csgs);
    stage(s, d.xforms, xforms);
    stage(s, d.tf_fwd, tf_f);
    stage(s, d.tf_inv, tf_i);
    stage(s, d.mats, mats);
    stage(s, d.media, media);
    d.has_media = media.empty() ? 0 : 1;
    // texture tables: Perlin values / permutations, image pixels
    std::vector<DPerlin> dper;
    std::vector<double> tf64;
    std::vector<int32_t> ti32;
    for (const HPerlin& hp : s->perlins) {
        DPerlin x;
        std::memset(&x, 0, sizeof(x));
        x.point_count = (int32_t)hp.d.point_count; x.vector = hp.d.vector; x.smooth = hp.d.smooth; x.type = hp.d.type;
        x.depth = (int32_t)hp.d.depth; x.scale = hp.d.scale;
        x.voff = (int32_t)tf64.size(); x.poff = (int32_t)ti32.size();
        tf64.insert(tf64.end(), hp.values.begin(), hp.values.end());
        ti32.insert(ti32.end(), hp.perms.begin(), hp.perms.end());
        dper.push_back(x);
    }
    std::vector<DImage> dimg;
    std::vector<uint8_t> tu8;
    for (const HImage& hi : s->images) {
        DImage x; x.w = hi.w; x.h = hi.h; x.off = tu8.size();
        tu8.insert(tu8.end(), hi.rgb.begin(), hi.rgb.end());
        dimg.push_back(x);
    }
    stage(s, d.perlins, dper);
    stage(s, d.tex_f64, tf64);
    stage(s, d.tex_i32, ti32);
    stage(s, d.images, dimg);
    stage(s, d.tex_u8, tu8);
    d.uv = 0;  // only the Image texture reads (u, v)
    for (const DMaterial& m : mats) if (m.tex_kind == RS_TEX_IMAGE) d.uv = 1;
    stage(s, d.lights, lights);
    d.n_lights = (int32_t)lights.size();
    d.root = root;
    d.default_mat = default_mat;
    d.ref_order = s->ref_order ? 1 : 0;
    for (int i = 0; i < 3; ++i) { d.bg_lo[i] = s->bg_lo[i]; d.bg_hi[i] = s->bg_hi[i]; }
    d.bg_lo[3] = d.bg_hi[3] = 1.0f;
    build_limg(s);
}

// rs_scene_commit / rs_scene_commit_devices: build once, then one replica per listed device
// (none: a host-only build whose tree can be inspected with rs_scene_get_info).
// devices == nullptr with n == 1: the current device (rs_scene_commit).
void commit(rs_scene* s, const int* devices, int n) {
    if (s->committed) throw Error(RS_E_STATE, "scene already committed");
    if (n < 0 || (n > 1 && !devices)) throw Error(RS_E_INVALID, "bad device list");
    build(s);  // scene errors (e.g. RS_E_NO_LIGHTS) before any device work
    int current = 0;
    if (n == 1 && !devices) {
        HIP_OK(hipGetDevice(&current));
        devices = &current;
    }
    int count = 0;
    if (n > 0) HIP_OK(hipGetDeviceCount(&count));
    for (int i = 0; i < n; ++i)
        if (devices[i] < 0 || devices[i] >= count) throw Error(RS_E_INVALID, "device ordinal out of range");
    int prev = 0;
    if (n > 0) HIP_OK(hipGetDevice(&prev));
    try {
        for (int i = 0; i < n; ++i) upload_replica(s, devices[i]);
        // peer access between distinct devices, for the frame-end row gather of rs_render_device
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) {
                if (devices[i] == devices[j]) continue;
                int can = 0;
                if (hipDeviceCanAccessPeer(&can, devices[i], devices[j]) == hipSuccess && can) {
                    (void)hipSetDevice(devices[i]);
                    (void)hipDeviceEnablePeerAccess(devices[j], 0);  // already enabled is fine
                    (void)hipGetLastError();
                }
            }
    } catch (...) {
        s->reps.clear();
        (void)hipSetDevice(prev);
        throw;
    }
    if (n > 0) HIP_OK(hipSetDevice(prev));
    s->committed = true;
}

// camera.rs:37-73 with CameraBuilder's aspect = width/height (camera.rs:384-397)
DCamera make_camera(const rs_camera_desc& c) {
    auto sub = [](const double* a, const double* b, double* o) { for (int i = 0; i < 3; ++i) o[i] = a[i] - b[i]; };
    auto len2 = [](const double* a) { return std::fma(a[2], a[2], std::fma(a[0], a[0], a[1] * a[1])); };
    auto unit = [&](const double* a, double* o) { double inv = 1.0 / std::sqrt(len2(a)); for (int i = 0; i < 3; ++i) o[i] = a[i] * inv; };
    auto cross = [](const double* a, const double* b, double* o) {
        double r[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
        o[0] = r[0]; o[1] = r[1]; o[2] = r[2];
    };
    const double aspect = (double)c.width / (double)c.height;
    const double theta = c.fov * (3.14159265358979323846 / 180.0);
    const double h = std::tan(theta / 2.0);
    const double vh = 2.0 * h * c.focus;
    const double vw = vh * aspect;
    double w[3], d[3], hu[3], vu[3], t[3];
    sub(c.look_at, c.look_from, d);
    unit(d, w);
    cross(w, c.vup, t); unit(t, hu);
    cross(hu, w, t); unit(t, vu);
    DCamera o;
    for (int i = 0; i < 3; ++i) {
        o.origin[i] = c.look_from[i];
        o.hf[i] = hu[i] * vw;
        o.vf[i] = vu[i] * vh;
        o.hu[i] = hu[i];
        o.vu[i] = vu[i];
    }
    for (int i = 0; i < 3; ++i) {  // look_from - U/2 - V/2 + focus*w  (Div<f64> = * (1/2))
        double half = 1.0 / 2.0;
        o.lb[i] = c.look_from[i] - o.hf[i] * half - o.vf[i] * half + w[i] * c.focus;
    }
    o.aperture = c.aperture;
    o.shutter = c.shutter;
    return o;
}

uint64_t splitmix64_h(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

// grow a device buffer; `owner` (a slot or a replica) is quiesced first: frames in flight may still
// use the old one
template <typename T, class Q>
void ensure(Q& owner, T*& p, size_t& cap, size_t n) {
    if (n <= cap) return;
    if (p) { owner.quiesce(); HIP_OK(hipFree(p)); }
    p = nullptr;
    cap = 0;
    HIP_OK(hipMalloc((void**)&p, n * sizeof(T)));
    cap = n;
}
// ensure() that reports an out-of-memory device as false (nothing held then) instead of throwing
template <typename T, class Q>
bool try_ensure(Q& owner, T*& p, size_t& cap, size_t n) {
    if (n <= cap) return true;
    if (p) { owner.quiesce(); HIP_OK(hipFree(p)); }
    p = nullptr;
    cap = 0;
    const hipError_t e = hipMalloc((void**)&p, n * sizeof(T));
    if (e == hipErrorOutOfMemory) {
        (void)hipGetLastError();
        p = nullptr;
        return false;
    }
    HIP_OK(e);
    cap = n;
    return true;
}

// Traversal-stack overflow for launches of at most `threads` grid threads: (stack_need - kStackMax)
// entries per thread (DScene::stk_ovf). Nothing is allocated when the tree fits the LDS stack.
void ensure_stack_overflow(const rs_scene* s, Replica& R, uint64_t threads) {
    const int extra = s->stack_need - kStackMin;  // rows for the smallest LDS part (rs_internal.h stack_lds)
    if (extra <= 0) { R.ds.stk_ovf = nullptr; return; }
    ensure(R, R.d_ovf, R.ovf_cap, (size_t)extra * threads);
    R.ds.stk_ovf = R.d_ovf;
}

// a static scene's path records carry (item, level) in ray_o.w (rs_kernels.hip store_path; RS_NO_TAGW: the tag
// array, for A/B)
uint32_t tag_in_ray(const SceneRef& s) {
#ifdef RS_NO_TAGW
    (void)s;
    return 0u;
#else
    return s.host->moving == 0 ? 1u : 0u;
#endif
}

// bytes of one path of a wavefront pool (carve_wf): two sets of 3 x 32 B records + the tag, an entry per class queue
// (the bounce-synchronous wavefront's hit array shares the queues' memory)
constexpr uint64_t kPathBytes = 2 * (3 * sizeof(D4) + sizeof(uint2)) + kWfsClasses * sizeof(QEnt);

// Path state of `lanes` lanes of capacity `cap` paths per set each (L.lane_ws[l], L.d_qptrs[l], L.qptr[l]).
// Returns false, with the slot holding no pool, when the device cannot allocate it (the caller shrinks the pool).
bool carve_wf(Slot& L, uint64_t cap, uint32_t lanes) {
    const size_t per = kPathBytes;
    const uint64_t c = (std::max<uint64_t>(cap, L.wf_cap) + 255) & ~(uint64_t)255;
    const size_t lane_bytes = (per * c + 16 * 256 + 8192 + 255) & ~(size_t)255;
    const bool fresh = c > L.wf_cap || lanes > L.wf_lanes;
    if (fresh) {
        if (L.d_wf) { L.quiesce(); HIP_OK(hipFree(L.d_wf)); }
        L.d_wf = nullptr;
        L.wf_cap = 0;
        L.wf_lanes = 0;
        L.wf_bytes = 0;
        const hipError_t e = hipMalloc(&L.d_wf, lane_bytes * lanes);
        if (e == hipErrorOutOfMemory) {
            (void)hipGetLastError();  // not sticky: clear it for the next call's checks
            L.d_wf = nullptr;
            return false;
        }
        HIP_OK(e);
        L.wf_cap = c;
        L.wf_lanes = lanes;
        L.wf_bytes = lane_bytes * lanes;
    }
    auto al = [](char* p) { return (char*)(((uintptr_t)p + 255) & ~(uintptr_t)255); };
    for (uint32_t l = 0; l < lanes; ++l) {
        char* p = (char*)L.d_wf + lane_bytes * l;
        WfState& w = L.lane_ws[l];
        for (int k = 0; k < 2; ++k) {
            WfSet& t = w.set[k];
            t.ray_o = (D4*)p; p += sizeof(D4) * c;
            t.ray_d = (D4*)p; p += sizeof(D4) * c;
            t.thr = (D4*)p; p += sizeof(D4) * c;
            t.tag = (uint2*)p; p = al(p + sizeof(uint2) * c);
        }
        w.hit = (double2*)p;  // (bounce-synchronous wavefront; the streaming one's queues below)
        QEnt* qp[kWfsClasses];
        for (int k = 0; k < kWfsClasses; ++k) { qp[k] = (QEnt*)p; p = al(p + sizeof(QEnt) * c); }
        L.d_qptrs[l] = (QEnt**)p;
        w.fetch = (uint32_t*)al(p + sizeof(qp));  // 1 KiB (kFetchCounters x kFetchStride words), zeroed by k_wf_gen
        w.heads = w.fetch + 256;                   // 2 KiB: 2 banks x 8 shards x 32 words
        if (fresh) HIP_OK(hipMemcpy(L.d_qptrs[l], qp, sizeof(qp), hipMemcpyHostToDevice));
        for (int k = 0; k < kWfsClasses; ++k) L.qptr[l][k] = qp[k];
        w.counts = nullptr;
        w.cap = (uint32_t)c;
    }
    return true;
}

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        HIP_OK(hipGetDevice(&prev));
        if (prev != dev) HIP_OK(hipSetDevice(dev));
    }
    ~DeviceGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

// Rows of the call's lattice (row_begin, row_end, row_step) that replica k of n renders: every n-th
// lattice row starting at the k-th, the interleave of render_rows (painter.rs:248) over devices.
struct RowSet {
    uint32_t begin = 0, end = 0, step = 1;
    uint32_t count() const { return begin < end ? (end - begin + step - 1) / step : 0; }
};
RowSet replica_rows(const rs_camera_desc* cam, const rs_render_settings* st, uint32_t k, uint32_t n) {
    RowSet r;
    const uint32_t H = cam->height;
    const uint32_t re = st->row_end ? std::min(st->row_end, H) : H;
    const uint32_t rstep = st->row_step ? st->row_step : 1;
    const uint64_t b = (uint64_t)st->row_begin + (uint64_t)k * rstep;
    r.end = re;
    r.begin = b < re ? (uint32_t)b : re;
    r.step = (uint32_t)std::min<uint64_t>((uint64_t)rstep * n, 0xFFFFFFFFull);
    return r;
}

// Streaming schedule of a frame. The frame's camera samples form batches of B items
// (whole sample planes; the last may be shorter), dealt to L lanes round robin: lane l streams batches
// l, l + L, ... through its own pool on its own stream, injecting Q samples per iteration. Lane-local
// item j of lane l is item j - m B of its m-th batch. Batch k may be accumulated once the lane's
// iteration done(k) (its last sample injected + depth - 1) has run; its radiance lives in buffer
// k % ring of the rad ring, which a batch may take over only after the batch `ring` earlier was
// accumulated (the lane waits for that accumulate).
struct LaneSched {
    std::vector<uint32_t> batch;        // global batch ids, in the lane's order
    uint64_t total = 0, Q = 0, T_inj = 0, T = 0, cap = 0;
    uint64_t cnt_off = 0;               // the lane's counter blocks in the frame's counter array (words)
    uint64_t B = 0, last_nb = 0;        // batch size, size of the lane's last batch
    uint32_t D = 0;
    bool finish = false;                // the last iteration traces every carried path to its end (k_wfs_finish)
    uint64_t nb(uint64_t m) const { return m + 1 == batch.size() ? last_nb : B; }
    uint64_t first_it(uint64_t m) const { return (m * B) / Q; }
    uint64_t done_it(uint64_t m) const {
        const uint64_t end = std::min((m + 1) * B, total);
        return std::min((end - 1) / Q + (D ? D - 1 : 0), T - 1);
    }
    uint32_t n_new(uint64_t t) const { return t < T_inj ? (uint32_t)std::min(Q, total - t * Q) : 0u; }
};
struct FrameSched {
    uint64_t B = 0;
    uint32_t n_batches = 0, lanes = 1, ring = 1;
    uint32_t nbpf = 0;                  // batches per frame (a multi-pass stream: frame k / nbpf, its batch k % nbpf)
    std::vector<uint64_t> keys;         // per frame: PathParams::key_base of its pass
    std::vector<LaneSched> lane;
    uint64_t n_counts = 0;              // counter words of all lanes
    uint64_t cap = 0;                   // pool records per set (the largest lane's)
};
// The enqueue order of a frame (render_enqueue walks it; make_sched dry-runs it to size the ring):
// iterations round robin over the lanes; after each, every accumulate whose batches are complete, in
// batch order. visit(l, t) for an iteration, acc(k) for an accumulate.
template <class FI, class FA>
void walk(const FrameSched& f, FI visit, FA acc) {
    std::vector<uint64_t> t(f.lanes, 0), m_done(f.lanes, 0);
    std::vector<char> done(f.n_batches, 0);
    uint32_t next_acc = 0;
    for (bool any = true; any;) {
        any = false;
        for (uint32_t l = 0; l < f.lanes; ++l) {
            const LaneSched& L = f.lane[l];
            if (t[l] >= L.T) continue;
            any = true;
            visit(l, t[l]);
            while (m_done[l] < L.batch.size() && L.done_it(m_done[l]) == t[l]) done[L.batch[m_done[l]++]] = 1;
            ++t[l];
            while (next_acc < f.n_batches && done[next_acc]) acc(next_acc++);
        }
    }
}
FrameSched make_sched(const rs_scene* s, uint64_t n_pix, uint32_t N, uint32_t D, uint32_t want_lanes, uint64_t pool,
                      uint32_t n_frames = 1) {
    FrameSched f;
    // batches: at most max_items_per_batch items, and at least one per lane; n_frames > 1 (the passes of one
    // multi-pass stream, one after the other): every frame whole batches of the same size
    uint32_t spb = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(N, s->max_items_per_batch / n_pix));
    spb = std::min(spb, std::max<uint32_t>(1, (N + want_lanes - 1) / want_lanes));
    if (n_frames > 1)
        while (N % spb) --spb;
    f.B = n_pix * spb;
    f.nbpf = (N + spb - 1) / spb;
    f.n_batches = f.nbpf * n_frames;
    f.lanes = std::max<uint32_t>(1, std::min(want_lanes, f.n_batches));
    f.lane.resize(f.lanes);
    const uint64_t frame_items = n_pix * N;
    for (uint32_t k = 0; k < f.n_batches; ++k) {
        LaneSched& L = f.lane[k % f.lanes];
        L.batch.push_back(k);
        const uint64_t nb = std::min(f.B, frame_items - (uint64_t)(k % f.nbpf) * f.B);
        L.total += nb;
        L.last_nb = nb;
    }
    for (LaneSched& L : f.lane) {
        L.B = f.B;
        L.D = D;
        // about 1/inject_div of the lane per iteration, at most a batch; the pool's bound, Q times the
        // iterations a path can span, must fit pool_paths
        const uint64_t Dm = std::max<uint32_t>(D, 1);
        uint64_t q = std::min<uint64_t>(f.B, std::max<uint64_t>(kBlock, (L.total + s->inject_div - 1) / s->inject_div));
        auto bound = [&](uint64_t qq) { return qq * std::min<uint64_t>(Dm, (L.total + qq - 1) / qq); };
        if (bound(q) > pool) q = std::min<uint64_t>(f.B, std::max<uint64_t>(kBlock, pool / Dm));
        L.Q = q;
        L.T_inj = (L.total + q - 1) / q;
        L.T = L.T_inj + (D ? D - 1 : 0);
        // the finish: after the last injection, finish_after wavefront iterations, then one launch that traces
        // every path still carried to its end (a depth-50 frame's last ~40 iterations carry a few thousand paths
        // each and cost their launch gaps and one traversal's latency apiece). Measured (finish_after 0 / 4 / 8 /
        // 12, profiles/r5/ab/finish_after_r5e.jsonl): example.sdl 800x500x64 8.51 / 10.63 / 8.46 / 8.01 ms, RTIOW
        // 1920x1080x64 47.96 / 58.54 / 46.52 / 44.54 ms; 12 / 16 / 24 (finish_after_r5f.jsonl): 8.03 / 7.62 / 7.77
        // and 44.30 / 44.06 / 44.73 ms -- but quadric.sdl (9 segments per sample: many paths
        // still alive, and the finish runs them one thread each at 2 waves) 113.6 / 182.5 / 157.8 / 144.7 ms, so
        // nest-2 scenes do not finish
        if (s->finish_after && s->scene_mode != kSmNest2 && L.T > L.T_inj + s->finish_after + 1) {
            L.finish = true;
            L.T = L.T_inj + s->finish_after + 1;
        }
        L.cap = bound(q);
        L.cnt_off = f.n_counts;
        f.n_counts += (L.T + 1) * kWfsStride;
        f.cap = std::max(f.cap, L.cap);
    }
    // ring: the most batches ever begun and not yet accumulated in the enqueue order
    std::vector<uint64_t> start(f.n_batches, UINT64_MAX), acc_at(f.n_batches, 0);
    uint64_t step = 0;
    walk(f, [&](uint32_t l, uint64_t t) {
             const LaneSched& L = f.lane[l];
             for (uint64_t m = 0; m < L.batch.size(); ++m)
                 if (L.first_it(m) == t && start[L.batch[m]] == UINT64_MAX) start[L.batch[m]] = step;
             ++step;
         },
         [&](uint32_t k) { acc_at[k] = step; });
    for (uint32_t k = 0; k < f.n_batches; ++k) {
        uint32_t live = 1;
        // per lane its batches start in order: count each lane's later batches begun before acc(k)
        for (uint32_t l = 0; l < f.lanes; ++l) {
            uint32_t j = k + 1 + (l + f.lanes - (k + 1) % f.lanes) % f.lanes;
            for (; j < f.n_batches && start[j] < acc_at[k]; j += f.lanes) ++live;
        }
        f.ring = std::max(f.ring, live);
    }
    if ((uint64_t)f.ring * f.B > 0xFFFFFFFFull) throw Error(RS_E_INVALID, "batch too large for the radiance ring (lower max_batch_items)");
    if (f.cap > 0xFFFFFFFFull - 1024) throw Error(RS_E_INVALID, "path pool too large");
    return f;
}

// One replica's share of a frame between enqueue and finish: multi-device renders enqueue every
// replica before waiting for any, so the devices run concurrently.
struct Pending {
    Replica* R = nullptr;
    Slot* L = nullptr;
    uint32_t rec_bytes = 104;       // a path record as the kernels write it (96: the tag in ray_o.w, tag_in_ray)
    hipStream_t stream = nullptr;   // the stream the frame ends on (the caller's, or the replica's own)
    bool empty = true;
    int kind = 0;                   // 0 megakernel, 1 bounce-synchronous wavefront, 2 streaming wavefront
    bool timed = false;             // per-kernel events; the frame runs alone
    bool counted = false;           // the queue counters are kept for render_finish (statistics)
    uint32_t n_pix = 0, N = 0, depth = 0, n_batches = 0, path_launches = 0, n_frames = 1;
    uint64_t n_chunks_total = 0;
    std::vector<LaneSched> lanes;               // streaming: the lanes' schedules
    std::vector<std::vector<uint32_t>> inj;     // streaming: camera samples injected per lane and iteration
    size_t ki = 0;
    std::vector<hipEvent_t> ev, kev;
    unsigned long long cnt[512];
    std::vector<uint32_t> qc;
    ~Pending() {
        for (auto& e : ev) (void)hipEventDestroy(e);
        for (auto& e : kev) (void)hipEventDestroy(e);
    }
};

// The pool (paths per lane and set) of a frame on slot L of replica R streaming on `lanes` lanes: the scene's bound,
// capped so that the pools of all the replica's frame slots take at most two thirds of the device memory (kPathBytes
// per path and lane; 288 GB holds three slots of 256 Mi paths on one lane). A pool size is scheduling only: frames do
// not depend on it (rs_host.cpp make_sched, tests/test_gpu_parity.py test_streaming_pool_and_async_bit_identical).
uint32_t frame_slots(const rs_scene* s);
uint64_t pool_limit(const rs_scene* s, const Replica& R, uint32_t lanes) {
    const uint64_t per = kPathBytes * std::max<uint32_t>(1, lanes);
    return std::min<uint64_t>(s->pool_paths, std::max<uint64_t>(kBlock, R.mem_total / 3 * 2 / (frame_slots(s) * per)));
}
// ... and what the device can give it now: the memory free at render time (hipMemGetInfo) plus the pool and radiance
// ring this slot already holds (freed before larger ones are allocated), shared with the replica's slots that have
// no pool yet, each keeping `other` bytes (the frame's radiance ring) and 1 GiB (accumulation, counters, kernel
// scratch) outside the pool. A caller that keeps other data on the device (a PyTorch caching allocator, another
// scene) then gets a smaller pool instead of an allocation failure. Queried only when the slot has to allocate.
uint64_t pool_limit_free(const rs_scene* s, const Replica& R, const Slot& L, uint32_t lanes, uint64_t other) {
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
        (void)hipGetLastError();
        return kBlock;
    }
    const uint32_t n_slots = frame_slots(s);
    uint32_t empty = 0;
    for (uint32_t k = 0; k < n_slots; ++k)
        if (&R.slots[k] == &L || !R.slots[k].d_wf) ++empty;
    const uint64_t mine = (L.d_wf ? L.wf_bytes : 0) + L.rad_cap * sizeof(double);
    const uint64_t share = ((uint64_t)free_b + mine) / 10 * 9 / std::max<uint32_t>(1, empty);
    const uint64_t keep = other + (1ull << 30);
    return std::max<uint64_t>(kBlock, (share > keep ? share - keep : 0) / (kPathBytes * std::max<uint32_t>(1, lanes)));
}
// give back a slot's path pool and radiance ring (before a smaller pool is tried)
void release_pool(Slot& L) {
    if (!L.d_wf && !L.d_rad) return;
    L.quiesce();
    if (L.d_wf) HIP_OK(hipFree(L.d_wf));
    if (L.d_rad) HIP_OK(hipFree(L.d_rad));
    L.d_wf = nullptr; L.wf_cap = 0; L.wf_lanes = 0; L.wf_bytes = 0;
    L.d_rad = nullptr; L.rad_cap = 0;
}

// samples of a frame from which the spheres mode shades in two launches (rs_scene::shade_split)
#ifndef RS_SPLIT_SHADE_MIN  // (2 Mi, so the N = 8 row share's 3.2 M-sample frames split too: share 0.943 -> 0.968 ms
#define RS_SPLIT_SHADE_MIN (8ull << 20)  // with three frame slots, profiles/r5/ab/split_shade_min_r6o.txt)
#endif
constexpr uint64_t kSplitShadeMin = RS_SPLIT_SHADE_MIN;

// Frame slots a replica cycles through (render_enqueue takes slot next_slot % frame_slots): one for trees
// whose traversal stack spills to the replica's shared HBM overflow array, else frames_in_flight. Callers
// that keep several frames (bands) in flight must not exceed it: two frames in one slot share its counters.
uint32_t frame_slots(const rs_scene* s) {
    if (s->stack_need > stack_lds(s->scene_mode)) return 1u;
    return std::max<uint32_t>(1, std::min(kMaxSlots, s->frames_in_flight));
}

void validate_render(const rs_scene* s, const rs_camera_desc* cam, const rs_render_settings* st) {
    if (!cam || !st) throw Error(RS_E_INVALID, "null argument");
    if (!s->committed) throw Error(RS_E_STATE, "scene not committed");
    if (s->reps.empty()) throw Error(RS_E_STATE, "scene committed without devices (host-only build)");
    if (cam->width == 0 || cam->height == 0) throw Error(RS_E_INVALID, "empty image");
    if (st->mode < RS_MODE_AUTO || st->mode > RS_MODE_WAVEFRONT) throw Error(RS_E_INVALID, "unknown render mode");
    const uint32_t re = st->row_end ? std::min(st->row_end, cam->height) : cam->height;
    const uint32_t rstep = st->row_step ? st->row_step : 1;
    if (st->row_begin < re && (uint64_t)((re - st->row_begin + rstep - 1) / rstep) * cam->width > 0xFFFFFFFFull)
        throw Error(RS_E_INVALID, "frame too large");
}

hipStream_t lane_stream(Slot& L, uint32_t l) {
    if (!L.lane[l]) HIP_OK(hipStreamCreateWithFlags(&L.lane[l], hipStreamNonBlocking));
    if (!L.join_ev[l]) HIP_OK(hipEventCreateWithFlags(&L.join_ev[l], hipEventDisableTiming));
    return L.lane[l];
}

// The camera samples lane ln injects at iteration t (InjParams).
InjParams inj_params(const FrameSched& f, const LaneSched& ln, uint64_t t) {
    InjParams I{};
    I.n_new = ln.n_new(t);
    if (I.n_new) {
        const uint64_t j0 = t * ln.Q, m = j0 / f.B;
        const uint32_t k = ln.batch[m];
        I.jb0 = (uint32_t)(j0 - m * f.B);
        I.nb0 = (uint32_t)ln.nb(m);
        I.nb1 = m + 1 < ln.batch.size() ? (uint32_t)ln.nb(m + 1) : 0u;
        I.g0 = (uint64_t)(k % f.nbpf) * f.B;
        I.key0 = f.keys[k / f.nbpf];
        I.rad0 = (uint32_t)((k % f.ring) * f.B);
        if (m + 1 < ln.batch.size()) {
            const uint32_t k1 = ln.batch[m + 1];
            I.g1 = (uint64_t)(k1 % f.nbpf) * f.B;
            I.key1 = f.keys[k1 / f.nbpf];
            I.rad1 = (uint32_t)((k1 % f.ring) * f.B);
        }
    }
    return I;
}

// Enqueue the rows `rows` of the frame on replica R (its device must be current): camera samples ->
// wavefront (streaming or bounce-synchronous) or megakernel -> ordered accumulation -> into_color into
// d_out (W*H RGBA on R's device), the last step on `S`, the stream the frame ends on. The path work
// runs on one of R's frame slots. Nothing here waits for the device.
// n_frames > 1 (streaming scene modes, no mask): the passes st->pass + f, f < n_frames, of the frame as one sample
// stream -- pass f + 1's camera samples enter the path pool while pass f's paths drain -- into outs[f] (d_out
// unused); every frame is the one a call for its pass alone renders (the samples' keys, rad slots and the
// accumulation order are the same). The frames before the last are written from the slot's accumulate stream,
// after `outs_after` (the caller's work on S before the call).
void render_enqueue(const rs_scene* s, Replica& R, const rs_camera_desc* cam, const rs_render_settings* st,
                    RowSet rows, const uint8_t* d_mask, float* d_out, hipStream_t S, Pending& P, bool timed,
                    bool counted, uint32_t n_frames = 1, float* const* outs = nullptr, hipEvent_t outs_after = nullptr) {
    P.R = &R;
    P.stream = S;
    P.timed = timed;
    P.counted = counted = counted || timed;
    const uint32_t n_rows = rows.count();
    if (n_rows == 0) return;
    P.empty = false;
    // one frame at a time for trees whose traversal stack spills to the replica's shared HBM overflow
    const bool ext_spill = s->stack_need > stack_lds(s->scene_mode);
    const uint32_t n_slots = frame_slots(s);
    Slot& L = R.slots[R.next_slot % n_slots];
    R.next_slot = (R.next_slot + 1) % n_slots;
    P.L = &L;
    const hipStream_t L0 = lane_stream(L, 0);
    if (!L.free_ev) HIP_OK(hipEventCreateWithFlags(&L.free_ev, hipEventDisableTiming));
    if (!L.entry_ev) HIP_OK(hipEventCreateWithFlags(&L.entry_ev, hipEventDisableTiming));
    // the slot's previous frame must be done with its buffers; the caller's earlier work must be
    // done when the kernels read the caller's memory (the mask); a timed frame runs alone
    if (L.free_rec) HIP_OK(hipStreamWaitEvent(L0, L.free_ev, 0));
    if (d_mask || timed) {
        HIP_OK(hipEventRecord(L.entry_ev, S));
        HIP_OK(hipStreamWaitEvent(L0, L.entry_ev, 0));
    }
    if (timed)
        for (Slot& o : R.slots)
            if (&o != &L && o.free_rec) HIP_OK(hipStreamWaitEvent(L0, o.free_ev, 0));

    const bool wavefront = st->mode != RS_MODE_MEGAKERNEL;
    const bool streaming = wavefront && streaming_mode(s->scene_mode);
    if (n_frames > 1 && (!streaming || d_mask || !outs || !outs_after))
        throw Error(RS_E_INVALID, "multi-pass stream: streaming scenes, no mask");
    const uint32_t W = cam->width, H = cam->height;
    const uint32_t n_pix = (uint32_t)((uint64_t)n_rows * W);
    const uint32_t sq = (uint32_t)std::floor(std::sqrt((double)st->samples));  // painter.rs:110-118
    const uint32_t N = sq * sq;
    const uint32_t D = st->depth;

    DCamera dc = make_camera(*cam);
    PathParams pp{};
    pp.n_pix_local = n_pix; pp.width = W; pp.height = H; pp.row_begin = rows.begin; pp.row_step = rows.step;
    pp.sqrt_spp = sq; pp.depth = D;
    pp.key_base = splitmix64_h(splitmix64_h(st->seed) ^ (uint64_t)st->pass);
    pp.mask = d_mask;
    FinalParams fp;
    fp.n_pix_local = n_pix; fp.width = W; fp.row_begin = rows.begin; fp.row_step = rows.step; fp.n_samples = N;
    fp.gamma = st->gamma; fp.mask = d_mask;

    const uint32_t spb = N ? (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(N, s->max_items_per_batch / n_pix)) : 0;
    const uint32_t n_batches = spb ? (N + spb - 1) / spb : 0;
    ensure(L, L.d_acc, L.acc_cap, (size_t)3 * n_pix);
    if (!L.d_cnt) HIP_OK(hipMalloc((void**)&L.d_cnt, 512 * sizeof(unsigned long long)));
    // launch grids: grid-stride kernels over at most these many blocks (shading grids and the
    // streaming extend: 64 per CU; 8 -> 64 measured 9.22 -> 9.12 ms on the bench frame in round 2)
    const uint32_t wide = (uint32_t)std::max(1, R.n_cu * 64);
    // the streaming extend: one block per 256 paths (a grid-stride loop over fewer blocks waits at the
    // queue barriers for its slowest wave, batch after batch); a bounded grid where the traversal stack
    // spills to the HBM overflow array, which is sized by grid threads
    const uint32_t ext_cap = ext_spill ? wide : 0xFFFFFFFFu;
    const uint32_t ext_blocks = (uint32_t)std::max(1, R.n_cu * std::max(1, R.ext_bpc));
    const uint32_t shade_blocks = (uint32_t)std::max(1, R.n_cu * std::max(1, R.shade_bpc));
    ensure_stack_overflow(s, R, (uint64_t)std::max(std::max(ext_blocks, shade_blocks), wide) * kBlock);
    const SceneRef ds = R.ref();
    P.rec_bytes = tag_in_ray(ds) ? 96u : 104u;
    const int sm = s->scene_mode;

    auto new_ev = [&]() { hipEvent_t e; HIP_OK(hipEventCreate(&e)); return e; };
    // the frame's end on S: join L0 into S, then the last accumulate there (it writes the caller's frame)
    auto join_to_S = [&]() {
        if (S == L0) return;
        HIP_OK(hipEventRecord(L.join_ev[0], L0));
        HIP_OK(hipStreamWaitEvent(S, L.join_ev[0], 0));
    };
    size_t ki = 0;
    uint32_t path_launches = 0;
    size_t n_counts = 0;

    if (N == 0) {  // no samples: into_color of 0 / 0 (NaN, or 0 with the mask) for every lattice pixel
        HIP_OK(hipMemsetAsync(L.d_acc, 0, (size_t)3 * n_pix * sizeof(double), L0));
        join_to_S();
        HIP_OK(launch_finalize(L.d_acc, d_out, fp, S));
    } else if (streaming) {
        const uint32_t want = ext_spill ? 1u : std::min<uint32_t>(kMaxLanes, s->stream_lanes);
        uint64_t pool = pool_limit(s, R, want);
        FrameSched f = make_sched(s, n_pix, N, D, want, pool, n_frames);
        auto rad_n = [&]() { return (size_t)3 * f.ring * f.B; };
        // the smallest pool a frame is scheduled on: 64 Ki camera samples per iteration (or the whole frame); below
        // that the iterations (and their counter blocks) multiply, and the render reports the device as full
        const uint64_t pool_min = std::min<uint64_t>(f.cap, (uint64_t)65536 * std::max<uint32_t>(D, 1));
        if (f.cap > L.wf_cap || f.lanes > L.wf_lanes || rad_n() > L.rad_cap) {
            // the slot allocates: as much as the device has free
            const uint64_t fp = std::max(pool_min, pool_limit_free(s, R, L, want, rad_n() * sizeof(double)));
            if (fp < pool) { pool = fp; f = make_sched(s, n_pix, N, D, want, pool, n_frames); }
        }
        // an allocation that still fails (memory taken meanwhile): both buffers back, half the pool
        while (!carve_wf(L, f.cap, f.lanes) || !try_ensure(L, L.d_rad, L.rad_cap, rad_n())) {
            release_pool(L);
            if (pool <= pool_min) throw Error(RS_E_NOMEM, "device memory exhausted: no room for the frame's path pool");
            pool = std::max<uint64_t>(pool_min, pool / 2);
            f = make_sched(s, n_pix, N, D, want, pool, n_frames);
        }
        f.keys.resize(n_frames);
        for (uint32_t k = 0; k < n_frames; ++k)
            f.keys[k] = splitmix64_h(splitmix64_h(st->seed) ^ (uint64_t)(st->pass + k));
        n_counts = f.n_counts;
        uint32_t* const prev_counts = L.d_counts;
        ensure(L, L.d_counts, L.counts_cap, n_counts);
        if (L.d_counts != prev_counts) L.counts_clean = 0;
        if (n_counts > L.counts_clean) HIP_OK(hipMemsetAsync(L.d_counts, 0, n_counts * sizeof(uint32_t), L0));
        L.counts_clean = 0;
        // Carried-extend grids. Without history a carried launch takes a block per 256 of the paths injected in the
        // last depth - 1 iterations (the bound on what it can carry), though from the second bounce on it carries a
        // few of them (bench frame: 28 % at t = 2, 3 % at t = 7): the empty blocks only read the count and leave, but
        // their dispatch costs a launch some microseconds. A frame of the same shape as one completed earlier takes
        // that frame's count of the iteration + 25 % + 16 Ki paths (blocks grid-stride over what exceeds it, so the
        // frame never depends on the estimate). The counts reach pinned host memory at the end of each frame
        // (Slot::h_hist) and are read here without waiting (bench frame 6.47 -> 6.39 ms with a fixed cap,
        // profiles/r6/ab/carried_cap_r6g1.txt).
        uint64_t sig = splitmix64_h(((uint64_t)n_pix << 32) ^ N) ^ splitmix64_h(((uint64_t)D << 40) ^ ((uint64_t)f.lanes << 32) ^ n_frames);
        std::vector<size_t> hoff(f.lanes, 0);
        size_t hwords = 0;
        for (uint32_t l = 0; l < f.lanes; ++l) {
            const LaneSched& ln = f.lane[l];
            sig = splitmix64_h(sig ^ ln.Q ^ (ln.T << 40) ^ (ln.total << 1) ^ (uint64_t)ln.finish);
            hoff[l] = hwords;
            hwords += ln.T;
        }
        for (Slot& o : R.slots) {
            if (!o.hist_pending) continue;
            const hipError_t q = hipEventQuery(o.hist_ev);
            if (q == hipSuccess) {
                o.hist_pending = false;
                R.hist.assign(o.h_hist, o.h_hist + o.hist_words);
                R.hist_sig = o.hist_sig;
            } else {
                (void)hipGetLastError();  // hipErrorNotReady: not an error here
                if (q != hipErrorNotReady) HIP_OK(q);
            }
        }
#ifdef RS_NO_GRID_HINT  // (dev A/B: every carried launch over a block per 256 paths of the window)
        const bool hint = false;
#else
        const bool hint = R.hist_sig == sig && R.hist.size() == hwords;
#endif
        if (L.hist_cap < hwords) {
            if (L.h_hist) { HIP_OK(hipEventSynchronize(L.hist_ev)); HIP_OK(hipHostFree(L.h_hist)); L.h_hist = nullptr; }
            HIP_OK(hipHostMalloc((void**)&L.h_hist, hwords * sizeof(uint32_t)));
            L.hist_cap = hwords;
            L.hist_pending = false;
        }
        if (!L.hist_ev) HIP_OK(hipEventCreateWithFlags(&L.hist_ev, hipEventDisableTiming));
        // every lane and the accumulate stream start after L0's dependencies and the counter reset
        hipStream_t ls[kMaxLanes] = {L0};
        for (uint32_t l = 1; l < f.lanes; ++l) ls[l] = lane_stream(L, l);
        if (!L.acc_stream) HIP_OK(hipStreamCreateWithFlags(&L.acc_stream, hipStreamNonBlocking));
        if (!L.fork_ev) HIP_OK(hipEventCreateWithFlags(&L.fork_ev, hipEventDisableTiming));
        HIP_OK(hipEventRecord(L.fork_ev, L0));
        for (uint32_t l = 1; l < f.lanes; ++l) HIP_OK(hipStreamWaitEvent(ls[l], L.fork_ev, 0));
        HIP_OK(hipStreamWaitEvent(L.acc_stream, L.fork_ev, 0));
        if (n_frames > 1) HIP_OK(hipStreamWaitEvent(L.acc_stream, outs_after, 0));
        // per batch: its paths are done (recorded on its lane) / it has been accumulated (acc stream)
        while (L.bev.size() < 2 * (size_t)f.n_batches) {
            hipEvent_t e;
            HIP_OK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            L.bev.push_back(e);
        }
        auto done_ev = [&](uint32_t k) { return L.bev[2 * (size_t)k]; };
        auto acc_ev = [&](uint32_t k) { return L.bev[2 * (size_t)k + 1]; };
        // (a multi-pass stream's iterations carry paths and inject camera samples: two launches, each part at its own
        // occupancy -- 30 share frames of the bench frame 0.971 -> 0.909 ms, profiles/r6/passes)
        const bool split = ext_split(sm) || s->ext_split || n_frames > 1;
        // lean / heavy shading launches (spheres mode; nest modes with an LDS image) pay one more launch tail per
        // iteration: worth it on full frames (bench 7.16 -> 7.09 ms), not on small ones (the N = 8 row share, 3.2 M
        // samples: 1.013 -> 1.066 ms)
        const bool split_shade = s->shade_split && (uint64_t)n_pix * N >= kSplitShadeMin;
        size_t n_ext = 0;
        for (const LaneSched& ln : f.lane) n_ext += ln.T * (split ? 2 : 1);
        P.kev.assign(timed ? 2 * n_ext : 0, nullptr);
        for (auto& e : P.kev) e = new_ev();
        P.ev.assign(timed ? 2 : 0, nullptr);  // path_ms: the frame's iterations
        for (auto& e : P.ev) e = new_ev();
        if (timed) HIP_OK(hipEventRecord(P.ev[0], L0));
        P.lanes.assign(f.lane.begin(), f.lane.end());
        // per lane: the samples injected by its last depth - 1 iterations (a bound on the paths it
        // carries into the next one), its next batch to be done, and the injections per iteration
        std::vector<uint64_t> window(f.lanes, 0), m_done(f.lanes, 0);
        std::vector<std::vector<uint32_t>> inj(f.lanes);
        for (uint32_t l = 0; l < f.lanes; ++l) inj[l].assign(f.lane[l].T, 0u);
        walk(f,
             [&](uint32_t l, uint64_t t) {
                 const LaneSched& ln = f.lane[l];
                 const hipStream_t cs = ls[l];
                 WfState WS = L.lane_ws[l];
                 WS.tagw = tag_in_ray(ds);
                 WS.counts = L.d_counts + ln.cnt_off;
                 QEnt** qd = L.d_qptrs[l];
                 const uint32_t n_new = ln.n_new(t);
                 inj[l][t] = n_new;
                 InjParams I = inj_params(f, ln, t);
                 if (n_new) {
                     const uint64_t m = t * ln.Q / f.B;
                     // a batch taking over a ring buffer: after the batch `ring` earlier was accumulated
                     for (uint64_t mm = m; mm <= m + 1 && mm < ln.batch.size(); ++mm) {
                         const uint32_t kk = ln.batch[mm];
                         if (ln.first_it(mm) == t && kk >= f.ring) HIP_OK(hipStreamWaitEvent(cs, acc_ev(kk - f.ring), 0));
                     }
                 }
                 if (ln.finish && t + 1 == ln.T) {  // the finish: every carried path to its end, one launch
                     const uint32_t b = (uint32_t)std::min<uint64_t>(wide, (window[l] + kBlock - 1) / kBlock);
                     // timed with the extends: it traces the World::hit of every segment it runs (the statistics
                     // count them on this iteration), so the dominant kernel's time covers the frame's segments
                     if (timed) HIP_OK(hipEventRecord(P.kev[2 * ki], cs));
                     HIP_OK(launch_wfs_finish(ds, WS, (uint32_t)t, D, L.d_rad, std::max<uint32_t>(1, b), sm, cs));
                     if (timed) HIP_OK(hipEventRecord(P.kev[2 * ki + 1], cs));
                     ++ki;
                     ++path_launches;
                     window[l] = 0;
                     while (m_done[l] < ln.batch.size() && ln.done_it(m_done[l]) == t)
                         HIP_OK(hipEventRecord(done_ev(ln.batch[m_done[l]++]), cs));
                     return;
                 }
                 auto extend = [&](int part, uint64_t n_max) {
                     if (hint && part == kExtCarried) {
                         const uint64_t est = R.hist[hoff[l] + t];
                         n_max = std::min<uint64_t>(n_max, est + est / 4 + 64ull * kBlock);
                     }
                     const uint32_t b = (uint32_t)std::min<uint64_t>(ext_cap, (n_max + kBlock - 1) / kBlock);
                     if (!b) return;
                     HIP_OK(launch_wfs_extend(ds, dc, pp, WS, qd, (uint32_t)t, I, L.d_rad, b, part, sm, cs,
                                              timed ? P.kev[2 * ki] : nullptr, timed ? P.kev[2 * ki + 1] : nullptr));
                     ++ki;
                     ++path_launches;
                 };
                 // an iteration with only carried paths (or only camera samples) runs the kernel compiled for
                 // that part alone: nest-0 example.sdl 8.95 -> 8.41 ms; the spheres mode's carried part runs at 5
                 // waves (ext_min_waves), bench frame 7.58 -> 7.31 ms (profiles/r5/ab; at 4 waves its parts had
                 // measured 2.8 % slower than the merged kernel, profiles/r4/ab/part_pick)
                 if (split) {
                     extend(kExtCarried, window[l]);
                     extend(kExtCamera, n_new);
                 } else if (n_new == 0) {
                     extend(kExtCarried, window[l]);
                 } else if (window[l] == 0) {
                     extend(kExtCamera, n_new);
                 } else {
                     extend(kExtAll, window[l] + n_new);
                 }
                 if (D > 0) {
                     uint64_t n_sh = window[l] + n_new;  // the paths it may shade: at most the live ones
#ifndef RS_NO_SHADE_HINT  // (dev A/B)
                     if (hint) {
                         const uint64_t est = R.hist[hoff[l] + t];
                         n_sh = std::min<uint64_t>(n_sh, est + est / 4 + 64ull * kBlock + n_new);
                     }
#endif
                     const uint32_t b = (uint32_t)std::min<uint64_t>(wide, (n_sh + kBlock - 1) / kBlock);
                     HIP_OK(launch_wfs_shade_all(ds, WS, qd, s->class_mask, (uint32_t)t, D, L.d_rad, b,
                                                 split_shade, sm, cs));
                     ++path_launches;
                 }
                 // carried into t + 1: the samples injected by iterations t - depth + 2 .. t
                 window[l] += n_new;
                 if (D == 0) window[l] = 0;
                 else if (t + 1 >= D) window[l] -= inj[l][t + 1 - D];
                 while (m_done[l] < ln.batch.size() && ln.done_it(m_done[l]) == t)
                     HIP_OK(hipEventRecord(done_ev(ln.batch[m_done[l]++]), cs));
             },
             [&](uint32_t k) {
                 // batch k's samples have all finished: accumulate in sample order (the last batch on S,
                 // writing the frame and zeroing the counters for the next frame unless statistics read them;
                 // an earlier pass's last batch into its frame, on the accumulate stream)
                 const uint32_t fr = k / f.nbpf, kl = k % f.nbpf;
                 float* const out = n_frames > 1 ? outs[fr] : d_out;
                 const uint32_t planes = (uint32_t)(std::min<uint64_t>(f.B, (uint64_t)n_pix * N - (uint64_t)kl * f.B) / n_pix);
                 const double* rk = L.d_rad + (size_t)3 * (k % f.ring) * f.B;  // item-major radiance (put_rad)
                 if (k + 1 < f.n_batches) {
                     HIP_OK(hipStreamWaitEvent(L.acc_stream, done_ev(k), 0));
                     HIP_OK(launch_accumulate(rk, L.d_acc, n_pix, planes, kl == 0, kl + 1 == f.nbpf ? 1 : 0, fp, out,
                                              nullptr, 0, L.acc_stream));
                     HIP_OK(hipEventRecord(acc_ev(k), L.acc_stream));
                 } else {
                     HIP_OK(hipEventRecord(L.join_ev[0], L.acc_stream));
                     HIP_OK(hipStreamWaitEvent(S, L.join_ev[0], 0));
                     HIP_OK(hipStreamWaitEvent(S, done_ev(k), 0));
                     for (uint32_t l = 1; l < f.lanes; ++l) {  // (every lane's last iteration, for the counters)
                         HIP_OK(hipEventRecord(L.join_ev[l], ls[l]));
                         HIP_OK(hipStreamWaitEvent(S, L.join_ev[l], 0));
                     }
                     HIP_OK(hipEventRecord(L.fork_ev, L0));
                     HIP_OK(hipStreamWaitEvent(S, L.fork_ev, 0));
                     // the frame's carried counts (counter slot 0 of each lane's iterations) for later frames' grids,
                     // before the accumulate zeroes them
                     for (uint32_t l = 0; l < f.lanes; ++l)
                         HIP_OK(hipMemcpy2DAsync(L.h_hist + hoff[l], sizeof(uint32_t), L.d_counts + f.lane[l].cnt_off,
                                                 kWfsStride * sizeof(uint32_t), sizeof(uint32_t), f.lane[l].T,
                                                 hipMemcpyDeviceToHost, S));
                     HIP_OK(hipEventRecord(L.hist_ev, S));
                     L.hist_pending = true;
                     L.hist_sig = sig;
                     L.hist_words = hwords;
                     const size_t nz = counted ? 0 : n_counts;
                     HIP_OK(launch_accumulate(rk, L.d_acc, n_pix, planes, kl == 0, 1, fp, out, L.d_counts,
                                              (uint32_t)nz, S));
                     L.counts_clean = nz;
                 }
             });
        P.inj = std::move(inj);
        if (timed) HIP_OK(hipEventRecord(P.ev[1], S));
    } else {
        // bounce-synchronous wavefront (flat / rich scenes) or megakernel: per batch of spb sample planes
        ensure(L, L.d_rad, L.rad_cap, (size_t)3 * n_pix * spb);
        // Wavefront lanes (rs_scene_set_lanes, default 2): a batch's chunks go round-robin to lane streams
        // and run concurrently, so one lane's launch tails and small late-bounce launches overlap the
        // other's work. Chunks are whole sample planes when the batch allows (camera-ray tile order,
        // gen_perm). Scenes whose traversal stack spills to HBM keep one lane (the overflow array is
        // shared by blockIdx).
        const uint32_t want = (wavefront && !ext_spill) ? std::min<uint32_t>(kMaxLanes, s->wf_lanes) : 1u;
        uint32_t lanes = want;
        uint64_t chunk = 0, n_chunks_total = 0;
        auto plan = [&](uint64_t pool) {  // chunks of at most `pool` paths per lane
            lanes = want;
            chunk = std::max<uint64_t>(kBlock, std::min<uint64_t>(pool, (uint64_t)n_pix * spb));
            if (lanes > 1) {
                const uint64_t planes = (spb + lanes - 1) / lanes;
                const uint64_t split = std::max<uint64_t>(kBlock, spb >= lanes ? (uint64_t)n_pix * planes
                                                                               : ((uint64_t)n_pix * spb + lanes - 1) / lanes);
                chunk = std::min(chunk, split);
            }
            n_chunks_total = 0;
            for (uint32_t s0 = 0; s0 < N; s0 += spb) n_chunks_total += ((uint64_t)n_pix * std::min(spb, N - s0) + chunk - 1) / chunk;
            if (n_chunks_total < lanes) lanes = std::max<uint32_t>(1, (uint32_t)n_chunks_total);
        };
        uint64_t pool = pool_limit(s, R, want);
        plan(pool);
        hipStream_t ls[kMaxLanes] = {L0};
        if (wavefront) {
            const uint64_t pool_min = std::min<uint64_t>(chunk, 1ull << 20);  // chunks of at least 1 Mi paths
            if (chunk > L.wf_cap || lanes > L.wf_lanes) {  // the slot allocates: as much as the device has free
                const uint64_t fp = std::max(pool_min, pool_limit_free(s, R, L, want, L.rad_cap * sizeof(double)));
                if (fp < pool) plan(pool = fp);  // (the slot's radiance buffer, allocated above, stays)
            }
            while (!carve_wf(L, chunk, lanes)) {
                if (pool <= pool_min) throw Error(RS_E_NOMEM, "device memory exhausted: no room for the frame's path pool");
                plan(pool = std::max<uint64_t>(pool_min, pool / 2));
            }
            n_counts = (size_t)n_chunks_total * (D + 1);
            uint32_t* const prev_counts = L.d_counts;
            ensure(L, L.d_counts, L.counts_cap, n_counts);
            if (L.d_counts != prev_counts) L.counts_clean = 0;
            for (uint32_t l = 1; l < lanes; ++l) ls[l] = lane_stream(L, l);
            if (lanes > 1 && !L.fork_ev) HIP_OK(hipEventCreateWithFlags(&L.fork_ev, hipEventDisableTiming));
        }
        P.ev.assign(timed ? 2 * (size_t)n_batches : 0, nullptr);
        for (auto& e : P.ev) e = new_ev();
        P.kev.assign(timed ? 2 * (wavefront ? (size_t)n_chunks_total * D : n_batches) : 0, nullptr);
        for (auto& e : P.kev) e = new_ev();
        if (!wavefront || timed) HIP_OK(hipMemsetAsync(L.d_cnt, 0, 512 * sizeof(unsigned long long), L0));
        if (n_counts > L.counts_clean) HIP_OK(hipMemsetAsync(L.d_counts, 0, n_counts * sizeof(uint32_t), L0));
        L.counts_clean = 0;
        uint32_t bi = 0;
        uint64_t chunk_i = 0;
        for (uint32_t s0 = 0; s0 < N; s0 += spb, ++bi) {
            const uint32_t nb = std::min(spb, N - s0);
            pp.s0 = s0;
            pp.n_items = (uint64_t)n_pix * nb;
            if (timed) HIP_OK(hipEventRecord(P.ev[2 * bi], L0));
            if (!wavefront) {
                if (timed) HIP_OK(hipEventRecord(P.kev[2 * ki], L0));
                HIP_OK(launch_path_mega(ds, dc, pp, sm, L.d_rad, L.d_cnt, wide, L0));
                if (timed) HIP_OK(hipEventRecord(P.kev[2 * ki + 1], L0));
                ++ki;
                ++path_launches;
            } else {
                if (lanes > 1) {  // fork: the lane streams start after what L0 holds
                    HIP_OK(hipEventRecord(L.fork_ev, L0));
                    for (uint32_t l = 1; l < lanes; ++l) HIP_OK(hipStreamWaitEvent(ls[l], L.fork_ev, 0));
                }
                uint32_t lane = 0;
                for (uint64_t c0 = 0; c0 < pp.n_items; c0 += chunk, ++chunk_i, lane = (lane + 1) % lanes) {
                    const uint32_t n = (uint32_t)std::min<uint64_t>(chunk, pp.n_items - c0);
                    WfState WS = L.lane_ws[lane];
                    WS.tagw = tag_in_ray(ds);
                    WS.counts = L.d_counts + chunk_i * (D + 1);
                    const hipStream_t cs = ls[lane];
                    // a pixel mask: k_wf_gen compacts the live samples into set 0's shards (counts from zero)
                    if (pp.mask) HIP_OK(hipMemsetAsync(WS.heads, 0, 8 * 32 * sizeof(uint32_t), cs));
                    HIP_OK(launch_wf_gen(dc, pp, WS, c0, n, L.d_rad, cs));
                    ++path_launches;
                    for (uint32_t b = 0; b < D; ++b) {
                        if (timed) HIP_OK(hipEventRecord(P.kev[2 * ki], cs));
                        // meshes: one block per 256 paths (C5 49.6 -> 48.1 ms), at most 64 per CU where the tree
                        // spills its stack to HBM (the overflow array is sized for that grid; a grid of resident
                        // blocks only, grid-striding, made the C5 extend 35 % slower); the rich mode a bounded grid
                        const uint32_t bn = (n + kBlock - 1) / kBlock;
                        // flat scenes on the 4-wide tree: the persistent extend (k_wf_extend_dyn), one resident grid
                        const uint32_t eb = sm == kSmFlat ? (flat_dyn(ds) ? std::min(ext_blocks, bn)
                                                                          : ext_spill ? std::min(wide, bn) : bn)
                                                          : std::min(ext_blocks, bn);
                        HIP_OK(launch_wf_extend(ds, WS, b, eb, sm, cs));
                        if (timed) HIP_OK(hipEventRecord(P.kev[2 * ki + 1], cs));
                        ++ki;
                        HIP_OK(launch_wf_shade(ds, WS, b, D, pp.n_items, L.d_rad,
                                               std::min(sm == kSmFlat ? wide : shade_blocks, (n + kBlock - 1) / kBlock),
                                               sm, cs));
                        path_launches += 2;
                    }
                }
                if (lanes > 1) {  // join: L0 continues after every lane's chunks
                    for (uint32_t l = 1; l < lanes; ++l) {
                        HIP_OK(hipEventRecord(L.join_ev[l], ls[l]));
                        HIP_OK(hipStreamWaitEvent(L0, L.join_ev[l], 0));
                    }
                }
            }
            if (timed) HIP_OK(hipEventRecord(P.ev[2 * bi + 1], L0));
            const bool last = s0 + spb >= N;
            if (!last) {
                HIP_OK(launch_accumulate(L.d_rad, L.d_acc, n_pix, nb, s0 == 0, 0, fp, d_out, nullptr, 0, L0));
            } else {
                // the last batch's accumulate finishes the frame (into_color) and, when no statistics
                // read the queue counters afterwards, zeroes them for the next frame (no memset launch)
                join_to_S();
                const size_t nz = (wavefront && !counted) ? n_counts : 0;
                HIP_OK(launch_accumulate(L.d_rad, L.d_acc, n_pix, nb, s0 == 0, 1, fp, d_out, L.d_counts,
                                         (uint32_t)nz, S));
                L.counts_clean = nz;
            }
        }
        P.n_chunks_total = n_chunks_total;
    }
    HIP_OK(hipEventRecord(L.free_ev, S));
    L.free_rec = true;
    P.kind = !wavefront ? 0 : streaming ? 2 : 1;
    P.n_frames = n_frames;
    P.n_pix = n_pix;
    P.N = N;
    P.depth = D;
    P.n_batches = n_batches;
    P.ki = ki;
    P.path_launches = path_launches;
}

// Wait for replica P's share and add its statistics into *stats (which the caller zeroed).
void render_finish(const rs_scene* s, Pending& P, rs_render_stats* stats) {
    if (P.empty) return;
    if (!P.counted || !stats) { HIP_OK(hipStreamSynchronize(P.stream)); return; }
    Slot& L = *P.L;
    // a timed frame: the counters after everything on its stream; a counted (untimed) one, whose stream may
    // already carry later frames in other slots (rs_render_rows' bands): the caller has waited for this
    // frame, so its slot's counters are final and are read on the slot's own lane stream
    const hipStream_t cs = P.timed ? P.stream : L.lane[0];
    HIP_OK(hipMemcpyAsync(P.cnt, L.d_cnt, sizeof(P.cnt), hipMemcpyDeviceToHost, cs));
    size_t words = 0;
    if (P.N > 0 && P.kind == 2)
        for (const LaneSched& ln : P.lanes) words = std::max<size_t>(words, ln.cnt_off + (ln.T + 1) * kWfsStride);
    if (P.N > 0 && P.kind == 1) words = (size_t)P.n_chunks_total * (P.depth + 1);
    P.qc.assign(words, 0u);
    if (words) HIP_OK(hipMemcpyAsync(P.qc.data(), L.d_counts, words * sizeof(uint32_t), hipMemcpyDeviceToHost, cs));
    HIP_OK(hipStreamSynchronize(cs));
    double path_ms = 0.0;
    for (size_t b = 0; b + 1 < P.ev.size(); b += 2) {
        float ms = 0;
        HIP_OK(hipEventElapsedTime(&ms, P.ev[b], P.ev[b + 1]));
        path_ms += ms;
    }
    double kernel_ms = 0.0;
    for (size_t k = 0; P.timed && k < P.ki; ++k) {  // (a counted, untimed frame has no kernel events)
        float ms = 0;
        HIP_OK(hipEventElapsedTime(&ms, P.kev[2 * k], P.kev[2 * k + 1]));
        kernel_ms += ms;
    }
    const uint64_t items = (uint64_t)P.n_pix * P.N * P.n_frames;
    uint64_t seg = 0, kbytes = 0;
    if (P.kind == 0) {
        for (int i = 0; i < 256; ++i) seg += P.cnt[i];
        stats->kernel_id = RS_KERNEL_PATH_MEGA;
        kbytes = 24ull * items;  // radiance out, 3 x f64 per sample
    } else if (P.kind == 1) {
        // segments = sum over chunks and bounces of the extend queue lengths; the extend reads a ray
        // (2 x 32 B records) and writes a hit (16 B) per segment
        for (uint64_t c = 0; c < P.n_chunks_total; ++c)
            for (uint32_t b = 0; b < P.depth; ++b) seg += P.qc[c * (P.depth + 1) + b];
#ifdef RS_DEV_KNOBS
        if (s->dump_iters)
            for (uint32_t b = 0; b < P.depth; ++b) {
                uint64_t nb = 0;
                for (uint64_t c = 0; c < P.n_chunks_total; ++c) nb += P.qc[c * (P.depth + 1) + b];
                std::fprintf(stderr, "bounce %2u: %11llu paths\n", b, (unsigned long long)nb);
            }
#endif
        stats->kernel_id = RS_KERNEL_WF_EXTEND;
        kbytes = 80ull * seg;
    } else {
        // the streaming extend's library byte model, per iteration: ray records in (64 B)
        // per carried path; the queue entry with the hit (16 B) per shaded segment; the record out (96 B + item
        // + level) per live camera sample (written after its traversal for the ones that go on to shading:
        // an upper bound); radiance out (24 B) per path ending in extend, + its throughput record and item
        // in (36 B); radiance out for masked samples
        for (size_t l = 0; l < P.lanes.size(); ++l)
            for (uint64_t t = 0; t < P.lanes[l].T; ++t) {
                const uint32_t* q = &P.qc[P.lanes[l].cnt_off + t * kWfsStride];
                uint64_t live_new = 0, shaded = 0;
                for (uint32_t k = 0; k < kStatLines; ++k) live_new += q[cix(kCntStat0 + (int)k)];
                for (int k = 0; k < kWfsClasses; ++k) shaded += q[cix(1 + k)];
                const uint64_t old = q[cix(0)], live = old + live_new;
                if (P.lanes[l].finish && t + 1 == P.lanes[l].T) {
                    // the finish: its carried paths' first segments and (stat lines) the ones after; a record in
                    // (104 B) and a radiance out (24 B) per path
                    seg += live;
                    kbytes += 128ull * old;
                    continue;
                }
                const uint64_t dead_new = P.inj[l][t] - live_new;
                const uint64_t ended = live - shaded;
                seg += live;
                kbytes += 64ull * old + 16ull * shaded + (uint64_t)P.rec_bytes * live_new + 60ull * ended + 24ull * dead_new;
#ifdef RS_DEV_KNOBS
                if (s->dump_iters) {
                    const uint32_t* qn = q + kWfsStride;  // the next set's runs
                    std::fprintf(stderr, "iter lane %zu t %3llu: carried %9llu (front %9u back %9u) camera %9llu shaded %9llu"
                                 " [%u %u %u %u %u] ended %9llu -> next front %9u back %9u\n", l, (unsigned long long)t,
                                 (unsigned long long)old, q[cix(kCntFront)], q[cix(kCntBack)], (unsigned long long)live_new,
                                 (unsigned long long)shaded, q[cix(1)], q[cix(2)], q[cix(3)], q[cix(4)], q[cix(5)],
                                 (unsigned long long)ended, qn[cix(kCntFront)], qn[cix(kCntBack)]);
                }
#endif
            }
        stats->kernel_id = RS_KERNEL_WFS_EXTEND;
    }
    stats->path_ms += path_ms;
    stats->launches += P.path_launches;
    stats->kernel_launches += (uint32_t)P.ki;
    stats->kernel_ms += kernel_ms;
    stats->kernel_bytes += kbytes;
    stats->segments += seg;
    stats->tree_arity = s->tree_arity;
    stats->samples += items;  // masked-out pixels included (they trace nothing)
}

// copy rows `rows` of a W-wide RGBA f32 frame between two buffers of the same layout
hipError_t copy_rows(float* dst, const float* src, uint32_t W, RowSet rows, hipMemcpyKind kind, hipStream_t st) {
    const uint32_t n = rows.count();
    if (n == 0) return hipSuccess;
    const size_t row_bytes = (size_t)W * 4 * sizeof(float);
    const size_t off = (size_t)rows.begin * W * 4;
    return hipMemcpy2DAsync(dst + off, row_bytes * rows.step, src + off, row_bytes * rows.step, row_bytes, n, kind, st);
}

// rs_render_device: replica 0 renders its rows straight into d_out, its frame ending on the caller's
// stream; every other replica renders into a frame of its own device (its slot's) ending on its own
// stream and copies its rows into d_out.
void render_frame_device(rs_scene* s, const rs_camera_desc* cam, const rs_render_settings* st, const uint8_t* d_mask,
                         float* d_out, hipStream_t stream, rs_render_stats* stats) {
    if (!d_out) throw Error(RS_E_INVALID, "null argument");
    validate_render(s, cam, st);
    rs_render_stats acc{};
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t n = (uint32_t)s->reps.size();
    const size_t npx = (size_t)cam->width * cam->height;
    std::vector<std::unique_ptr<Pending>> P(n);
    std::vector<hipEvent_t> done(n, nullptr);
    hipEvent_t entry = nullptr;  // what the caller queued on `stream` before this call (mask fill, d_out use)
    try {
        if (n > 1) {
            DeviceGuard g(s->reps[0]->device);
            HIP_OK(hipEventCreateWithFlags(&entry, hipEventDisableTiming));
            HIP_OK(hipEventRecord(entry, stream));
        }
        for (uint32_t k = 0; k < n; ++k) {
            Replica& R = *s->reps[k];
            P[k].reset(new Pending());
            const RowSet rows = replica_rows(cam, st, k, n);
            DeviceGuard g(R.device);
            if (k == 0) {
                render_enqueue(s, R, cam, st, rows, d_mask, d_out, stream, *P[k], stats != nullptr, false);
                continue;
            }
            if (rows.count() == 0) continue;
            // the replica's stream reads d_mask and writes d_out: order it after the caller's work
            HIP_OK(hipStreamWaitEvent(R.stream, entry, 0));
            // this frame's copies of the mask and the frame live in R's next slot (the slot render_enqueue
            // picks): its previous frame must be done with them
            const uint32_t n_slots = frame_slots(s);
            Slot& L = R.slots[R.next_slot % n_slots];
            if (L.free_rec) HIP_OK(hipStreamWaitEvent(R.stream, L.free_ev, 0));
            ensure(L, L.d_out, L.out_cap, npx * 4);
            const uint8_t* m = nullptr;
            if (d_mask) {
                ensure(L, L.d_mask, L.mask_cap, npx);
                HIP_OK(hipMemcpyAsync(L.d_mask, d_mask, npx, hipMemcpyDefault, R.stream));
                m = L.d_mask;
            }
            render_enqueue(s, R, cam, st, rows, m, L.d_out, R.stream, *P[k], stats != nullptr, false);
            HIP_OK(copy_rows(d_out, L.d_out, cam->width, rows, hipMemcpyDefault, R.stream));
            HIP_OK(hipEventRecord(L.free_ev, R.stream));  // the copy read the slot's frame
            HIP_OK(hipEventCreateWithFlags(&done[k], hipEventDisableTiming));
            HIP_OK(hipEventRecord(done[k], R.stream));
        }
        {
            DeviceGuard g(s->reps[0]->device);
            for (uint32_t k = 1; k < n; ++k)
                if (done[k]) HIP_OK(hipStreamWaitEvent(stream, done[k], 0));
        }
        if (stats) {  // without stats the call returns once everything is enqueued (asynchronous)
            for (uint32_t k = 0; k < n; ++k) {
                DeviceGuard g(s->reps[k]->device);
                render_finish(s, *P[k], &acc);
            }
            DeviceGuard g(s->reps[0]->device);
            HIP_OK(hipStreamSynchronize(stream));
        }
    } catch (...) {
        for (uint32_t k = 0; k < n; ++k)  // drain what was enqueued before the buffers go away
            if (P[k] && P[k]->R) { DeviceGuard g(P[k]->R->device); (void)hipDeviceSynchronize(); }
        for (hipEvent_t e : done) if (e) (void)hipEventDestroy(e);
        if (entry) (void)hipEventDestroy(entry);
        throw;
    }
    for (hipEvent_t e : done) if (e) (void)hipEventDestroy(e);
    if (entry) (void)hipEventDestroy(entry);
    acc.tree_arity = s->tree_arity;
    acc.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (stats) *stats = acc;
}

// rs_render_device_passes: passes st->pass + k into d_outs[k]. One replica, a streaming scene mode and a pass the
// stream pays for: multi-pass sample streams (render_enqueue's n_frames); otherwise a render_frame_device per pass.
// Measured, 30 passes of RTIOW per call against 30 asynchronous one-pass calls (ms per pass, profiles/r6/passes):
//   800x500x64 depth 8: 6.39 / 6.52 (stream), its rows 0::8 0.891 / 0.919; 400x250x16 0.492 / 0.502, rows 0::8
//   0.163 / 0.139; 200x125x16 0.202 / 0.197, rows 0::8 0.136 / 0.104; depth 50: 800x500x64 7.84 / 8.04, rows 0::8
//   1.256 / 1.064 -- the stream pays where a pass's late iterations are a large part of its time (small passes, or
//   deep ones of a few million samples), and costs 2-3 % on passes that fill the GPU by themselves.
bool passes_stream_pays(uint64_t items, uint32_t depth) {
    return items <= (1ull << 20) || (depth >= 16 && items <= (8ull << 20));
}
void render_passes_device(rs_scene* s, const rs_camera_desc* cam, const rs_render_settings* st, uint32_t n,
                          float* const* d_outs, hipStream_t stream, rs_render_stats* stats) {
    if (n && !d_outs) throw Error(RS_E_INVALID, "null argument");
    for (uint32_t k = 0; k < n; ++k)
        if (!d_outs[k]) throw Error(RS_E_INVALID, "null argument");
    validate_render(s, cam, st);
    const auto t0 = std::chrono::steady_clock::now();
    rs_render_stats acc{};
    const uint32_t sq = (uint32_t)std::floor(std::sqrt((double)st->samples));
    const RowSet rows = replica_rows(cam, st, 0, 1);
    const bool stream_all = n > 1 && s->reps.size() == 1 && st->mode != RS_MODE_MEGAKERNEL &&
                            streaming_mode(s->scene_mode) && sq > 0 && rows.count() > 0 &&
                            s->passes_stream != 2 &&
                            (s->passes_stream == 1 ||
                             passes_stream_pays((uint64_t)rows.count() * cam->width * sq * sq, st->depth));
    if (!stream_all) {
        for (uint32_t k = 0; k < n; ++k) {
            rs_render_settings sk = *st;
            sk.pass = st->pass + k;
            rs_render_stats one{};
            render_frame_device(s, cam, &sk, nullptr, d_outs[k], stream, stats ? &one : nullptr);
            acc.samples += one.samples; acc.segments += one.segments; acc.path_ms += one.path_ms;
            acc.launches += one.launches; acc.kernel_launches += one.kernel_launches; acc.kernel_ms += one.kernel_ms;
            acc.kernel_bytes += one.kernel_bytes; acc.kernel_id = one.kernel_id;
        }
    } else {
        // contiguous groups of passes, one per frame slot, streamed concurrently (a single sample stream is one chain
        // of dependent launches: 12 share frames of the bench frame took 1.01 ms each as one stream, 1.25 as one-pass
        // frames on one slot, 0.885 as one-pass frames over three slots; profiles/r6/passes); one group when an
        // output pointer repeats (later passes overwrite earlier ones: their writes stay in pass order)
        Replica& R = *s->reps[0];
        DeviceGuard g(R.device);
        uint32_t groups = std::min<uint32_t>(frame_slots(s), n);
        {
            std::vector<float*> sorted(d_outs, d_outs + n);
            std::sort(sorted.begin(), sorted.end());
            if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end()) groups = 1;
        }
        std::vector<std::unique_ptr<Pending>> P(groups);
        hipEvent_t entry = nullptr;  // the caller's work on `stream` before the call: the earlier frames' writes wait
        try {
            HIP_OK(hipEventCreateWithFlags(&entry, hipEventDisableTiming));
            HIP_OK(hipEventRecord(entry, stream));
            for (uint32_t k = 0; k < groups; ++k) {
                const uint32_t lo = (uint32_t)((uint64_t)n * k / groups), hi = (uint32_t)((uint64_t)n * (k + 1) / groups);
                rs_render_settings sg = *st;
                sg.pass = st->pass + lo;
                P[k].reset(new Pending());
                render_enqueue(s, R, cam, &sg, rows, nullptr, d_outs[lo], stream, *P[k], stats != nullptr, false,
                               hi - lo, d_outs + lo, entry);
                if (stats) render_finish(s, *P[k], &acc);
            }
            if (stats) HIP_OK(hipStreamSynchronize(stream));
        } catch (...) {
            (void)hipDeviceSynchronize();  // drain what was enqueued before the buffers go away
            if (entry) (void)hipEventDestroy(entry);
            throw;
        }
        HIP_OK(hipEventDestroy(entry));
    }
    acc.tree_arity = s->tree_arity;
    acc.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (stats) *stats = acc;
}

// rs_render: every replica renders its rows into a frame on its own device on its own stream; the
// rows are copied back into the caller's buffer (rows outside the call's lattice keep their values).
void render_frame_host(rs_scene* s, const rs_camera_desc* cam, const rs_render_settings* st, const uint8_t* mask,
                       float* out, rs_render_stats* stats) {
    if (!out) throw Error(RS_E_INVALID, "null argument");
    validate_render(s, cam, st);
    rs_render_stats acc{};
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t n = (uint32_t)s->reps.size();
    const size_t npx = (size_t)cam->width * cam->height;
    std::vector<std::unique_ptr<Pending>> P(n);
    std::vector<RowSet> rows(n);
    std::vector<Slot*> slot(n, nullptr);
    try {
        for (uint32_t k = 0; k < n; ++k) {
            Replica& R = *s->reps[k];
            P[k].reset(new Pending());
            rows[k] = replica_rows(cam, st, k, n);
            if (rows[k].count() == 0) continue;
            DeviceGuard g(R.device);
            const uint32_t n_slots = frame_slots(s);
            Slot& L = R.slots[R.next_slot % n_slots];
            slot[k] = &L;
            if (L.free_rec) HIP_OK(hipStreamWaitEvent(R.stream, L.free_ev, 0));
            ensure(L, L.d_out, L.out_cap, npx * 4);
            const uint8_t* m = nullptr;
            if (mask) {
                ensure(L, L.d_mask, L.mask_cap, npx);
                HIP_OK(hipMemcpyAsync(L.d_mask, mask, npx, hipMemcpyHostToDevice, R.stream));
                m = L.d_mask;
            }
            render_enqueue(s, R, cam, st, rows[k], m, L.d_out, R.stream, *P[k], stats != nullptr, false);
        }
        for (uint32_t k = 0; k < n; ++k) {
            if (rows[k].count() == 0) continue;
            Replica& R = *s->reps[k];
            DeviceGuard g(R.device);
            HIP_OK(copy_rows(out, slot[k]->d_out, cam->width, rows[k], hipMemcpyDeviceToHost, R.stream));
            HIP_OK(hipEventRecord(slot[k]->free_ev, R.stream));
            render_finish(s, *P[k], &acc);
            HIP_OK(hipStreamSynchronize(R.stream));
        }
    } catch (...) {
        for (uint32_t k = 0; k < n; ++k)
            if (P[k] && P[k]->R) { DeviceGuard g(P[k]->R->device); (void)hipDeviceSynchronize(); }
        throw;
    }
    acc.tree_arity = s->tree_arity;
    acc.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (stats) *stats = acc;
}

// rs_render_rows: the frame's row lattice in bands, each band a frame of its own on the replicas'
// frame slots (band b on replica b % n), up to frames_in_flight bands in flight per replica; each
// band's rows are copied to pinned host memory on the replica's stream, and once a band's copy is
// complete its rows are handed to the callback -- from the calling thread, in band order, while the
// later bands are traced (painter.rs:214's register_pixels as rows finish), then the sentinel.
void render_frame_rows(rs_scene* s, const rs_camera_desc* cam, const rs_render_settings* st, const uint8_t* mask,
                       float* out, uint32_t bands, rs_row_callback cb, void* user, rs_render_stats* stats) {
    if (!out || !cb) throw Error(RS_E_INVALID, "null argument");
    validate_render(s, cam, st);
    rs_render_stats acc{};
    const auto t0 = std::chrono::steady_clock::now();
    const uint32_t n = (uint32_t)s->reps.size();
    const uint32_t W = cam->width, H = cam->height;
    const size_t npx = (size_t)W * H;
    const uint32_t rb = st->row_begin, re = st->row_end ? std::min(st->row_end, H) : H;
    const uint32_t step = st->row_step ? st->row_step : 1;
    const uint32_t n_rows = rb < re ? (re - rb + step - 1) / step : 0;
    if (bands == 0) bands = 16;
    const uint32_t per = std::max<uint32_t>(1, (n_rows + bands - 1) / bands);
    const uint32_t n_bands = n_rows ? (n_rows + per - 1) / per : 0;
    // bands in flight per replica: one per frame slot (a band's statistics are read from its slot's counters,
    // so a second band in the same slot would overwrite them before render_finish reads them)
    const uint32_t ahead = frame_slots(s);
    float* pinned = nullptr;
    std::vector<std::unique_ptr<Pending>> P(n_bands);
    std::vector<hipEvent_t> copied(n_bands, nullptr);
    std::vector<RowSet> rows(n_bands);
    std::vector<uint8_t*> d_masks(n, nullptr);
    auto cleanup = [&]() {
        for (uint32_t k = 0; k < n; ++k) {
            DeviceGuard g(s->reps[k]->device);
            (void)hipStreamSynchronize(s->reps[k]->stream);
            if (d_masks[k]) (void)hipFree(d_masks[k]);
        }
        for (hipEvent_t e : copied) if (e) (void)hipEventDestroy(e);
        if (pinned) (void)hipHostFree(pinned);
    };
    try {
        HIP_OK(hipHostMalloc((void**)&pinned, npx * 4 * sizeof(float)));
        std::memcpy(pinned, out, npx * 4 * sizeof(float));  // rows off the lattice keep the caller's values
        if (mask)
            for (uint32_t k = 0; k < n; ++k) {  // the mask once per replica, read by all its bands
                DeviceGuard g(s->reps[k]->device);
                HIP_OK(hipMalloc((void**)&d_masks[k], npx));
                HIP_OK(hipMemcpyAsync(d_masks[k], mask, npx, hipMemcpyHostToDevice, s->reps[k]->stream));
            }
        auto enqueue = [&](uint32_t b) {
            Replica& R = *s->reps[b % n];
            DeviceGuard g(R.device);
            rs_render_settings bs = *st;
            bs.row_begin = rb + b * per * step;
            bs.row_end = (uint32_t)std::min<uint64_t>(re, (uint64_t)bs.row_begin + (uint64_t)per * step);
            bs.row_step = step;
            rows[b] = replica_rows(cam, &bs, 0, 1);
            const uint32_t n_slots = frame_slots(s);
            Slot& L = R.slots[R.next_slot % n_slots];
            if (L.free_rec) HIP_OK(hipStreamWaitEvent(R.stream, L.free_ev, 0));
            ensure(L, L.d_out, L.out_cap, npx * 4);
            P[b].reset(new Pending());
            render_enqueue(s, R, cam, &bs, rows[b], d_masks[b % n], L.d_out, R.stream, *P[b], false, stats != nullptr);
            HIP_OK(copy_rows(pinned, L.d_out, W, rows[b], hipMemcpyDeviceToHost, R.stream));
            HIP_OK(hipEventRecord(L.free_ev, R.stream));  // the copy read the slot's frame
            HIP_OK(hipEventCreateWithFlags(&copied[b], hipEventDisableTiming));
            HIP_OK(hipEventRecord(copied[b], R.stream));
        };
        for (uint32_t b = 0; b < std::min(n_bands, ahead * n); ++b) enqueue(b);
        for (uint32_t b = 0; b < n_bands; ++b) {
            {
                DeviceGuard g(s->reps[b % n]->device);
                HIP_OK(hipEventSynchronize(copied[b]));
                if (stats) render_finish(s, *P[b], &acc);  // the band's counts (untimed: bands overlap)
            }
            if (b + ahead * n < n_bands) enqueue(b + ahead * n);
            for (uint32_t y = rows[b].begin; y < rows[b].end; y += rows[b].step) {
                std::memcpy(out + (size_t)y * W * 4, pinned + (size_t)y * W * 4, (size_t)W * 4 * sizeof(float));
                cb(user, y, out + (size_t)y * W * 4, W);
            }
        }
    } catch (...) {
        cleanup();
        throw;
    }
    cleanup();
    cb(user, H, nullptr, 0);  // end-of-pass sentinel (painter.rs:332)
    acc.tree_arity = s->tree_arity;
    acc.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (stats) *stats = acc;
}

}  // namespace

namespace {
int run(const std::function<void()>& f) {
    try {
        f();
        return RS_OK;
    } catch (const Error& e) {
        g_last_error = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        g_last_error = "out of host memory";
        return RS_E_NOMEM;
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return RS_E_INVALID;
    }
}
rs_scene* S(rs_scene* s) {
    if (!s) throw Error(RS_E_INVALID, "null scene");
    return s;
}
}  // namespace

extern "C" {

int rs_abi_version(void) { return RS_ABI_VERSION; }
const char* rs_last_error(void) { return g_last_error.c_str(); }
int rs_device_count(int* count) {
    return run([&] { if (!count) throw Error(RS_E_INVALID, "null"); HIP_OK(hipGetDeviceCount(count)); });
}
uint64_t rs_stream_key(uint64_t seed, uint32_t pass, uint64_t pixel, uint32_t sample) {
    return splitmix64_h(splitmix64_h(splitmix64_h(splitmix64_h(seed) ^ (uint64_t)pass) ^ pixel) ^ (uint64_t)sample);
}
// Rng::medium_key + medium_uniform of rs_device.h
double rs_medium_uniform(const uint32_t st[4], uint32_t handle) {
    const uint64_t key = splitmix64_h((((uint64_t)st[1] << 32) | st[0]) ^ splitmix64_h(((uint64_t)st[3] << 32) | st[2]));
    return (double)splitmix64_h(key ^ splitmix64_h(0x6d656469756d2121ULL + (uint64_t)handle)) * 0x1p-64;
}

int rs_scene_create(rs_scene** out) {
    return run([&] {
        if (!out) throw Error(RS_E_INVALID, "null");
        rs_scene* s = new rs_scene();
#ifdef RS_DEV_KNOBS
        // dev builds only (raysnail_amd/csrc/Makefile `dev`: libraysnail_hip_dev.so): tuning overrides
        // for A/B runs; the shipped library reads no environment (rs_scene_set_* are the knobs)
        auto knob = [](const char* name, unsigned long long& v) {
            if (const char* e = std::getenv(name)) { const unsigned long long x = std::strtoull(e, nullptr, 10); if (x) v = x; }
        };
        unsigned long long v;
        v = s->max_items_per_batch; knob("RS_MAX_BATCH_ITEMS", v); s->max_items_per_batch = v;
        v = s->pool_paths; knob("RS_POOL_PATHS", v); s->pool_paths = v;
        v = s->inject_div; knob("RS_INJECT_DIV", v); s->inject_div = (uint32_t)v;
        if (const char* e = std::getenv("RS_FINISH_AFTER")) s->finish_after = (uint32_t)std::strtoul(e, nullptr, 10);
        v = s->wf_lanes; knob("RS_LANES", v); s->wf_lanes = (uint32_t)std::min<unsigned long long>(v, kMaxLanes);
        v = s->stream_lanes; knob("RS_SLANES", v); s->stream_lanes = (uint32_t)std::min<unsigned long long>(v, kMaxLanes);
        v = s->frames_in_flight; knob("RS_FRAMES", v); s->frames_in_flight = (uint32_t)std::min<unsigned long long>(v, kMaxSlots);
        v = 0; knob("RS_EXT_SPLIT", v); s->ext_split = v != 0;
        v = 0; knob("RS_SHADE_MERGED", v); if (v) s->shade_split = false;
        v = 0; knob("RS_DUMP_ITERS", v); s->dump_iters = v != 0;
        v = 0; knob("RS_PASSES_STREAM", v); s->passes_stream = (uint32_t)v;
#endif
        *out = s;
    });
}
int rs_scene_destroy(rs_scene* s) {
    return run([&] { delete s; });
}
int rs_material(rs_scene* s, const rs_material_desc* d, int32_t* id) {
    return run([&] {
        S(s);
        if (!d || !id) throw Error(RS_E_INVALID, "null argument");
        if (s->committed) throw Error(RS_E_STATE, "scene already committed");
        if (d->kind < RS_MAT_LAMBERTIAN || d->kind > RS_MAT_BLINN_PHONG) throw Error(RS_E_INVALID, "unknown material kind");
        if (d->texture.kind < RS_TEX_SOLID || d->texture.kind > RS_TEX_IMAGE) throw Error(RS_E_INVALID, "unknown texture kind");
        if (d->texture.kind == RS_TEX_PERLIN && (d->texture.data < 0 || (size_t)d->texture.data >= s->perlins.size()))
            throw Error(RS_E_INVALID, "texture refers to an unknown rs_perlin id");
        if (d->texture.kind == RS_TEX_IMAGE && (d->texture.data < 0 || (size_t)d->texture.data >= s->images.size()))
            throw Error(RS_E_INVALID, "texture refers to an unknown rs_image id");
        if (d->kind == RS_MAT_MIXED) {
            if (d->mix_a < 0 || (size_t)d->mix_a >= s->mdesc.size() || d->mix_b < 0 || (size_t)d->mix_b >= s->mdesc.size())
                throw Error(RS_E_INVALID, "mixed material refers to unknown ids");
        }
        *id = (int32_t)s->mdesc.size();
        s->mdesc.push_back(*d);
    });
}
int rs_perlin(rs_scene* s, const rs_perlin_desc* d, int32_t* id) {
    return run([&] {
        S(s);
        if (!d || !id || !d->values || !d->perm_x || !d->perm_y || !d->perm_z) throw Error(RS_E_INVALID, "null argument");
        if (s->committed) throw Error(RS_E_STATE, "scene already committed");
        const uint32_t n = d->point_count;
        if (n == 0 || (n & (n - 1)) != 0 || n > (1u << 24)) throw Error(RS_E_INVALID, "point_count must be a power of two");
        if (d->smooth < RS_SMOOTH_NONE || d->smooth > RS_SMOOTH_HERMITE || d->type < RS_PERLIN_NORMAL ||
            d->type > RS_PERLIN_MARBLE || d->depth > 64)
            throw Error(RS_E_INVALID, "bad Perlin smooth / type / depth");
        HPerlin hp;
        hp.d = *d;
        hp.d.values = nullptr; hp.d.perm_x = hp.d.perm_y = hp.d.perm_z = nullptr;
        hp.values.assign(d->values, d->values + (size_t)n * (d->vector ? 3 : 1));
        for (const uint32_t* perm : {d->perm_x, d->perm_y, d->perm_z})
            for (uint32_t i = 0; i < n; ++i) {
                if (perm[i] >= n) throw Error(RS_E_INVALID, "Perlin permutation entry out of range");
                hp.perms.push_back((int32_t)perm[i]);
            }
        *id = (int32_t)s->perlins.size();
        s->perlins.push_back(std::move(hp));
    });
}
int rs_image(rs_scene* s, const uint8_t* rgb, uint32_t width, uint32_t height, int32_t* id) {
    return run([&] {
        S(s);
        if (!rgb || !id) throw Error(RS_E_INVALID, "null argument");
        if (s->committed) throw Error(RS_E_STATE, "scene already committed");
        if (width == 0 || height == 0) throw Error(RS_E_INVALID, "empty image");
        HImage hi;
        hi.w = width; hi.h = height;
        hi.rgb.assign(rgb, rgb + (size_t)width * height * 3);
        *id = (int32_t)s->images.size();
        s->images.push_back(std::move(hi));
    });
}
int rs_constant_medium(rs_scene* s, uint32_t boundary, const float color[4], double density, uint32_t* out) {
    return run([&] {
        S(s)->check_handle(boundary);
        if (!color || !out) throw Error(RS_E_INVALID, "null argument");
        if (s->committed) throw Error(RS_E_STATE, "scene already committed");
        // ConstantMedium::new (constant.rs:29-39): material Isotropic(color), neg_inv_density = -1 / density
        rs_material_desc m;
        std::memset(&m, 0, sizeof(m));
        m.kind = RS_MAT_ISOTROPIC;
        m.texture.kind = RS_TEX_SOLID;
        for (int i = 0; i < 4; ++i) m.texture.even[i] = m.texture.odd[i] = color[i];
        m.texture.scale = 1.0; m.refractive = 1.0; m.multiplier = 1.0; m.mix_p = 0.5; m.phong_exponent = 1;
        HObj o; o.kind = PK_MEDIUM; o.a = (int32_t)boundary;
        o.mat = (int32_t)s->mdesc.size();
        s->mdesc.push_back(m);
        o.p[0] = -1.0 / density;
        *out = s->add(o);
    });
}
int rs_sphere(rs_scene* s, const double c[3], double r, const double v[3], int32_t mat, uint32_t* out) {
    return run([&] {
        S(s)->check_mat(mat);
        if (!c || !out) throw Error(RS_E_INVALID, "null argument");
        HObj o; o.kind = PK_SPHERE; o.mat = mat;
        o.p[0] = c[0]; o.p[1] = c[1]; o.p[2] = c[2]; o.p[3] = r; o.p[4] = r * r;  // sphere.rs:35-43
        if (v) { o.p[5] = v[0]; o.p[6] = v[1]; o.p[7] = v[2]; }
        *out = s->add(o);
    });
}
int rs_aarect(rs_scene* s, int32_t plane, double k, double a0, double a1, double b0, double b1, int32_t mat, uint32_t* out) {
    return run([&] {
        S(s)->check_mat(mat);
        if (!out) throw Error(RS_E_INVALID, "null argument");
        if (!(a0 < a1) || !(b0 < b1)) throw Error(RS_E_INVALID, "AARectMetrics requires a0 < a1 and b0 < b1 (rect.rs:27-28)");
        HObj o; o.kind = PK_RECT; o.mat = mat;
        if (plane == RS_PLANE_XY) { o.ax[0] = 0; o.ax[1] = 1; o.ax[2] = 2; }
        else if (plane == RS_PLANE_XZ) { o.ax[0] = 0; o.ax[1] = 2; o.ax[2] = 1; }
        else if (plane == RS_PLANE_YZ) { o.ax[0] = 1; o.ax[1] = 2; o.ax[2] = 0; }
        else throw Error(RS_E_INVALID, "bad plane");
        o.p[0] = k; o.p[1] = a0; o.p[2] = a1; o.p[3] = b0; o.p[4] = b1;
        *out = s->add(o);
    });
}
int rs_box(rs_scene* s, const double p0[3], const double p1[3], int32_t mat, uint32_t* out) {
    return run([&] {
        S(s)->check_mat(mat);
        if (!p0 || !p1 || !out) throw Error(RS_E_INVALID, "null argument");
        HObj o; o.kind = PK_BOX; o.mat = mat;
        for (int i = 0; i < 3; ++i) { o.p[i] = std::fmin(p0[i], p1[i]); o.p[3 + i] = std::fmax(p0[i], p1[i]); }  // box.rs:40-45
        for (int i = 0; i < 3; ++i)
            if (!(o.p[i] < o.p[3 + i])) throw Error(RS_E_INVALID, "degenerate box: face metrics need a0 < a1 (rect.rs:27-28)");
        *out = s->add(o);
    });
}
int rs_quadric(rs_scene* s, const double q[10], int32_t mat, uint32_t* out) {
    return run([&] {
        S(s)->check_mat(mat);
        if (!q || !out) throw Error(RS_E_INVALID, "null argument");
        HObj o; o.kind = PK_QUADRIC; o.mat = mat;
        for (int i = 0; i < 10; ++i) o.p[i] = q[i];
        *out = s->add(o);
    });
}
int rs_triangles(rs_scene* s, const double* pos, const double* nrm, uint32_t n, int32_t mat, uint32_t* first) {
    return run([&] {
        S(s)->check_mat(mat);
        if (!pos || !first) throw Error(RS_E_INVALID, "null argument");
        *first = (uint32_t)s->objs.size();
        for (uint32_t i = 0; i < n; ++i) {
            HObj o; o.kind = PK_TRIANGLE; o.mat = mat;
            for (int j = 0; j < 9; ++j) o.p[j] = pos[9 * (size_t)i + j];
            for (int j = 0; j < 9; ++j) o.p[9 + j] = nrm ? nrm[9 * (size_t)i + j] : 0.0;
            s->add(o);
        }
    });
}
int rs_intersection(rs_scene* s, uint32_t a, uint32_t b, int32_t mat, uint32_t* out) {
    return run([&] {
        S(s)->check_mat(mat); s->check_handle(a); s->check_handle(b);
        if (!out) throw Error(RS_E_INVALID, "null argument");
        HObj o; o.kind = PK_AND; o.mat = mat; o.a = (int32_t)a; o.b = (int32_t)b;
        *out = s->add(o);
    });
}
int rs_difference(rs_scene* s, uint32_t a, uint32_t b, int32_t mat, uint32_t* out) {
    return run([&] {
        S(s)->check_mat(mat); s->check_handle(a); s->check_handle(b);
        if (!out) throw Error(RS_E_INVALID, "null argument");
        HObj o; o.kind = PK_SUB; o.mat = mat; o.a = (int32_t)a; o.b = (int32_t)b;
        *out = s->add(o);
    });
}
int rs_transformed(rs_scene* s, uint32_t obj, const rs_transform* st, uint32_t n, uint32_t* out) {
    return run([&] {
        S(s)->check_handle(obj);
        if (!out || (n && !st)) throw Error(RS_E_INVALID, "null argument");
        HObj o; o.kind = PK_XFORM; o.a = (int32_t)obj;
        for (uint32_t i = 0; i < n; ++i) {
            if (st[i].kind < RS_TF_TRANSLATE || st[i].kind > RS_TF_SCALE) throw Error(RS_E_INVALID, "unknown transform kind");
            o.tfs.push_back(st[i]);
        }
        o.mat = s->objs[obj].mat;  // TfFacade::material is never called upstream; kept for needs_lights
        *out = s->add(o);
    });
}
int rs_world_add(rs_scene* s, uint32_t h) {
    return run([&] { S(s)->check_handle(h); if (s->committed) throw Error(RS_E_STATE, "scene already committed"); s->world.push_back(h); });
}
int rs_lights_add(rs_scene* s, uint32_t h) {
    return run([&] { S(s)->check_handle(h); if (s->committed) throw Error(RS_E_STATE, "scene already committed"); s->lights.push_back(h); });
}
int rs_set_background(rs_scene* s, const float lo[3], const float hi[3]) {
    return run([&] {
        S(s);
        if (!lo || !hi) throw Error(RS_E_INVALID, "null argument");
        if (s->committed) throw Error(RS_E_STATE, "scene already committed");
        for (int i = 0; i < 3; ++i) { s->bg_lo[i] = lo[i]; s->bg_hi[i] = hi[i]; }
    });
}
int rs_set_time_range(rs_scene* s, double t0, double t1) {
    return run([&] {
        S(s);
        if (s->committed) throw Error(RS_E_STATE, "scene already committed");
        s->time0 = t0; s->time1 = t1;
    });
}
int rs_scene_commit(rs_scene* s) {
    return run([&] {
        commit(S(s), nullptr, 1);
    });
}
int rs_scene_commit_devices(rs_scene* s, const int* devices, int n) {
    return run([&] {
        if (n < 0 || (n > 0 && !devices)) throw Error(RS_E_INVALID, "bad device list");
        commit(S(s), devices, n);
    });
}
int rs_scene_set_lanes(rs_scene* s, uint32_t lanes) {
    return run([&] {
        if (!s) throw Error(RS_E_INVALID, "null argument");
        if (lanes > kMaxLanes) throw Error(RS_E_INVALID, "lanes must be 0 (defaults) or 1 .. 4");
        s->wf_lanes = lanes ? lanes : 2;
        s->stream_lanes = lanes ? lanes : 1;
    });
}
int rs_scene_set_frames_in_flight(rs_scene* s, uint32_t frames) {
    return run([&] {
        if (!s) throw Error(RS_E_INVALID, "null argument");
        if (frames < 1 || frames > kMaxSlots) throw Error(RS_E_INVALID, "frames in flight must be 1 .. 4");
        s->frames_in_flight = frames;
    });
}
int rs_scene_set_workspace(rs_scene* s, uint64_t max_batch_items, uint64_t pool_paths) {
    return run([&] {
        if (!s) throw Error(RS_E_INVALID, "null argument");
        if (max_batch_items && max_batch_items > (1ull << 31)) throw Error(RS_E_INVALID, "max_batch_items above 2^31");
        if (pool_paths && (pool_paths < kBlock || pool_paths > (1ull << 31))) throw Error(RS_E_INVALID, "pool_paths must be 256 .. 2^31");
        if (max_batch_items) s->max_items_per_batch = max_batch_items;
        if (pool_paths) s->pool_paths = pool_paths;
    });
}

int rs_scene_get_info(const rs_scene* s, rs_scene_info* out) {
    return run([&] {
        if (!s || !out) throw Error(RS_E_INVALID, "null argument");
        if (!s->committed) throw Error(RS_E_STATE, "scene not committed");
        std::memset(out, 0, sizeof(*out));
        out->tree_arity = s->tree_arity;
        out->ref_order = s->ref_order ? 1 : 0;
        out->scene_mode = s->scene_mode;
        out->tree_depth = s->tree_depth;
        out->stack_need = s->stack_need;
        out->stack_lds = stack_lds(s->scene_mode);
        out->n_nodes = s->n_nodes;
        out->n_objects = s->objs.size();
        out->n_world = s->world.size();
        out->n_devices = (int32_t)s->reps.size();
        out->class_mask = s->class_mask;
    });
}

int rs_render_device(rs_scene* s, const rs_camera_desc* cam, const rs_render_settings* st, const uint8_t* d_mask,
                     float* d_out, void* stream, rs_render_stats* stats) {
    return run([&] {
        render_frame_device(S(s), cam, st, d_mask, d_out, (hipStream_t)stream, stats);
    });
}

int rs_render_device_passes(rs_scene* s, const rs_camera_desc* cam, const rs_render_settings* st, uint32_t n_passes,
                            float* const* d_outs, void* stream, rs_render_stats* stats) {
    return run([&] {
        render_passes_device(S(s), cam, st, n_passes, d_outs, (hipStream_t)stream, stats);
    });
}

int rs_combine_pixels_device(float* d_acc, const float* d_new, uint64_t n_pixels, float pass, void* stream) {
    return run([&] {
        if (!d_acc || !d_new) throw Error(RS_E_INVALID, "null argument");
        HIP_OK(launch_combine(d_acc, d_new, n_pixels, pass, (hipStream_t)stream));
    });
}

int rs_noise_map_device(const float* d_rgba, uint32_t width, uint32_t height, float threshold, uint8_t* d_redo,
                        void* stream, rs_noise_stats* stats) {
    return run([&] {
        if (!d_rgba) throw Error(RS_E_INVALID, "null argument");
        if ((uint64_t)width * height > 0x7FFFFFFFull) throw Error(RS_E_INVALID, "frame too large");
        const hipStream_t st = (hipStream_t)stream;
        // [0] min bits, [1] max bits (non-negative floats order like their bit patterns), [2..3] count
        unsigned int* d = nullptr;
        HIP_OK(hipMalloc((void**)&d, 4 * sizeof(unsigned int)));
        unsigned int init[4];
        float fmin0 = 3.0f, fmax0 = 1.0f;  // raysnail.rs:396-397
        std::memcpy(&init[0], &fmin0, 4);
        std::memcpy(&init[1], &fmax0, 4);
        init[2] = init[3] = 0;
        hipError_t e = hipMemcpyAsync(d, init, sizeof(init), hipMemcpyHostToDevice, st);
        if (e == hipSuccess)
            e = launch_noise(d_rgba, (int)width, (int)height, threshold, d_redo, d,
                             reinterpret_cast<unsigned long long*>(d + 2), st);
        unsigned int out[4] = {0, 0, 0, 0};
        if (e == hipSuccess) e = hipMemcpyAsync(out, d, sizeof(out), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        (void)hipFree(d);
        HIP_OK(e);
        if (stats) {
            std::memcpy(&stats->min, &out[0], 4);
            std::memcpy(&stats->max, &out[1], 4);
            uint64_t c;
            std::memcpy(&c, &out[2], 8);
            stats->count = c;
        }
    });
}

int rs_noise_map(const float* rgba, uint32_t width, uint32_t height, float threshold, uint8_t* redo,
                 rs_noise_stats* stats) {
    return run([&] {
        if (!rgba) throw Error(RS_E_INVALID, "null argument");
        const size_t n = (size_t)width * height;
        float* d_px = nullptr;
        uint8_t* d_redo = nullptr;
        HIP_OK(hipMalloc((void**)&d_px, n * 4 * sizeof(float) + 16));
        hipError_t e = hipMalloc((void**)&d_redo, n + 16);
        if (e == hipSuccess) e = hipMemcpy(d_px, rgba, n * 4 * sizeof(float), hipMemcpyHostToDevice);
        int rc = RS_OK;
        if (e == hipSuccess) rc = rs_noise_map_device(d_px, width, height, threshold, d_redo, nullptr, stats);
        if (e == hipSuccess && rc == RS_OK && redo) e = hipMemcpy(redo, d_redo, n, hipMemcpyDeviceToHost);
        (void)hipFree(d_px);
        (void)hipFree(d_redo);
        HIP_OK(e);
        if (rc != RS_OK) throw Error(rc, g_last_error);
    });
}

int rs_probe_world_hit(rs_scene* s, const double* rays, uint32_t n, double tmin, double tmax, double* out) {
    return run([&] {
        S(s);
        if (!s->committed) throw Error(RS_E_STATE, "scene not committed");
        if (!rays || !out) throw Error(RS_E_INVALID, "null argument");
        if (s->reps.empty()) throw Error(RS_E_STATE, "scene committed without devices (host-only build)");
        Replica& R = *s->reps[0];
        DeviceGuard g(R.device);
        double *dr = nullptr, *dout = nullptr;
        HIP_OK(hipMalloc((void**)&dr, (size_t)n * 7 * sizeof(double) + 8));
        HIP_OK(hipMalloc((void**)&dout, (size_t)n * 13 * sizeof(double) + 8));
        HIP_OK(hipMemcpy(dr, rays, (size_t)n * 7 * sizeof(double), hipMemcpyHostToDevice));
        ensure_stack_overflow(s, R, ((uint64_t)n + kBlock - 1) / kBlock * kBlock);
        HIP_OK(launch_probe_hit(R.ref(), dr, n, tmin, tmax, dout, nullptr));
        HIP_OK(hipMemcpy(out, dout, (size_t)n * 13 * sizeof(double), hipMemcpyDeviceToHost));
        (void)hipFree(dr);
        (void)hipFree(dout);
    });
}

int rs_probe_samples(rs_scene* s, const rs_camera_desc* cam, const rs_render_settings* st, uint32_t x, uint32_t y,
                     uint32_t s0, uint32_t n, double* out) {
    return run([&] {
        S(s);
        if (!cam || !st || !out) throw Error(RS_E_INVALID, "null argument");
        if (!s->committed) throw Error(RS_E_STATE, "scene not committed");
        if (x >= cam->width || y >= cam->height) throw Error(RS_E_INVALID, "pixel outside the frame");
        const uint32_t sq = (uint32_t)std::floor(std::sqrt((double)st->samples));
        if ((uint64_t)s0 + n > (uint64_t)sq * sq) throw Error(RS_E_INVALID, "sample index beyond floor(sqrt(samples))^2");
        if (s->reps.empty()) throw Error(RS_E_STATE, "scene committed without devices (host-only build)");
        Replica& R = *s->reps[0];
        DeviceGuard g(R.device);
        PathParams pp{};
        pp.n_pix_local = cam->width * cam->height; pp.width = cam->width; pp.height = cam->height;
        pp.row_begin = 0; pp.row_step = 1; pp.sqrt_spp = sq; pp.depth = st->depth;
        pp.key_base = splitmix64_h(splitmix64_h(st->seed) ^ (uint64_t)st->pass);
        double* dout = nullptr;
        HIP_OK(hipMalloc((void**)&dout, (size_t)n * 4 * sizeof(double) + 8));
        ensure_stack_overflow(s, R, ((uint64_t)n + kBlock - 1) / kBlock * kBlock);
        HIP_OK(launch_probe_sample(R.ref(), make_camera(*cam), pp, s->scene_mode, x, y, s0, n, dout, nullptr));
        HIP_OK(hipMemcpy(out, dout, (size_t)n * 4 * sizeof(double), hipMemcpyDeviceToHost));
        (void)hipFree(dout);
    });
}

int rs_render_rows(rs_scene* s, const rs_camera_desc* cam, const rs_render_settings* st, const uint8_t* mask,
                   float* out_rgba, uint32_t bands, rs_row_callback cb, void* user, rs_render_stats* stats) {
    return run([&] {
        render_frame_rows(S(s), cam, st, mask, out_rgba, bands, cb, user, stats);
    });
}

int rs_render(rs_scene* s, const rs_camera_desc* cam, const rs_render_settings* st, const uint8_t* mask, float* out,
              rs_render_stats* stats) {
    return run([&] {
        render_frame_host(S(s), cam, st, mask, out, stats);
    });
}

}  // extern "C"
