/*
 * raysnail_hip.h — C-ABI of libraysnail_hip.so, the MI355X (gfx950) render path.
 *
 * This is the drop-in boundary for raysnail's per-pixel render path
 *   Painter::draw sample loop -> Camera::ray -> Hittable::hit (BVH) -> Material::scatter/emitted
 * (reference: src/camera.rs:261-287 TakePhotoSettings::shot_to_target, src/painter.rs:307-336
 * Painter::draw). The GPU cannot call a Rust closure, so the boundary sits at shot_to_target
 * level: the caller flattens World + Camera + settings into plain-old-data through the calls
 * below, then asks for a frame. Every entry point is extern "C", takes plain pointers and sizes,
 * returns an int status (0 = ok, <0 = error) and never throws or aborts across the ABI;
 * rs_last_error() returns a thread-local message for the last failure on the calling thread.
 *
 * Reference interfaces replaced (file:line in Varkalandar/raysnail @ 2024-10-08):
 *   rs_scene_create/destroy  World::new                      src/hittable/collection/world.rs:40-53
 *   rs_material              Lambertian/Metal/DiffuseMetal/Dielectric/DiffuseLight/MixedMaterial
 *                            constructors                      src/material/{lambertian.rs:29-35,
 *                            metal.rs:43-49 (DiffuseMetal), metal.rs:95-100 (Metal), dielectric.rs:38-53,
 *                            light.rs:17-28, mixed_material.rs:32-38, isotropic.rs:15-22,
 *                            blinn_phong.rs:19-28}; textures Color / Checker / Perlin / Image
 *                            src/prelude/color.rs:61-65, src/texture/checker.rs:16-18,
 *                            src/texture/noise.rs, src/texture/image.rs;
 *                            CommonMaterialSettings src/material/mod.rs:41-54
 *   rs_sphere                Sphere::new / with_speed         src/hittable/geometry/sphere.rs:35-48
 *   rs_aarect                AARect::new_xy/new_xz/new_yz     src/hittable/geometry/rect.rs:58-79
 *   rs_box                   Box::new                         src/hittable/geometry/box.rs:40-45
 *   rs_quadric               Quadric::new                     src/hittable/geometry/quadric.rs:46-61
 *   rs_triangles             Triangle::new + set_normals      src/hittable/geometry/triangle_mesh.rs:42-71
 *   rs_intersection          Intersection::new                src/hittable/csg/intersection.rs:33-39
 *   rs_difference            Difference::new                  src/hittable/csg/difference.rs:32-38
 *   rs_transformed           TfFacade::new + TransformStack   src/hittable/transform/tf_facade.rs:30-37,
 *                                                             transform.rs:16-127
 *   rs_constant_medium       ConstantMedium::new (+ Isotropic) src/hittable/medium/constant.rs:29-39,
 *                                                             src/material/isotropic.rs:15-22
 *   rs_perlin                Perlin::new/scale/smooth/turbulence/marble  src/texture/noise.rs:44-103
 *   rs_image                 Image::new (decoded pixels)      src/texture/image.rs:24-31
 *   rs_world_add             HittableList::add (world list)   src/hittable/collection/list.rs:29-33
 *   rs_lights_add            HittableList::add (lights list)  src/hittable/collection/list.rs:29-33
 *   rs_set_background        World background closure         examples/rtow_13_1.rs:38-41,
 *                                                             src/bin/raysnail.rs:364-367
 *   rs_render                TakePhotoSettings::shot_to_target src/camera.rs:261-287 (CameraBuilder
 *                            src/camera.rs:300-413; Painter src/painter.rs:69-336)
 *   rs_render_device         same, with the frame left in device memory (no PCIe in the timed region)
 *   rs_render_device_passes  the CLI pass loop's renders (no redo map)  src/bin/raysnail.rs:379-427, as one call
 *
 * Output layout is the reference's Vec<[f32;4]>: W*H RGBA float32, row-major, row 0 = top,
 * sqrt-gamma applied when gamma != 0, unclamped, alpha 1.0 for rendered pixels, [0,0,0,0] for
 * pixels whose mask byte is 0 (PixelController::calculate_pixel == false, src/painter.rs:204-210).
 * Rows outside [row_begin, row_end) or not on the row_step lattice are left untouched.
 *
 * Determinism contract (the reference has none: every FastRng is seeded from thread_rng,
 * src/prelude/random.rs:116-121). Sample s of pixel p (linear index y*W+x) draws from its own
 * XorShift128 stream, seeded with rand_core-0.6 seed_from_u64(rs_stream_key(seed, pass, p, s)).
 * Within a sample, draws follow the reference order exactly: render_pixel jitter x then y
 * (painter.rs:167-170), Camera::ray disk rejection + shutter time (camera.rs:77-85), then per
 * bounce of ray_color (camera.rs:156-255). thread_rng draws on the path are taken from the same
 * stream at the same point: Dielectric's Random::normal (dielectric.rs:72) as one gen(),
 * MixedMaterial's next_u32 (mixed_material.rs:44) as one next_u32(). ConstantMedium::hit's
 * Random::normal() (medium/constant.rs:63) is called inside world.hit, where the number of calls
 * depends on the traversal; it is therefore NOT taken from the stream but from a counter-free hash
 * of the stream's state at the start of the segment and the medium's handle (rs_medium_uniform),
 * so every test of one medium within one world.hit sees the same draw, on every backend.
 */
#ifndef RAYSNAIL_HIP_H
#define RAYSNAIL_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RS_ABI_VERSION 6

/* ---- status codes ---- */
#define RS_OK             0
#define RS_E_INVALID     -1  /* bad argument / handle */
#define RS_E_NO_LIGHTS   -2  /* a pdf material exists but the lights list is empty (ref: % 0 panic, list.rs:51) */
#define RS_E_HIP         -3  /* HIP runtime error */
#define RS_E_STATE       -4  /* call not allowed in this state (e.g. render before commit) */
#define RS_E_UNSUPPORTED -5  /* construct outside what the GPU path implements */
#define RS_E_NOMEM       -6

/* ---- textures (src/prelude/color.rs:61-65, src/texture/{checker.rs:21-30, noise.rs, image.rs}) ---- */
#define RS_TEX_SOLID   0
#define RS_TEX_CHECKER 1
#define RS_TEX_PERLIN  2  /* data = rs_perlin id; Color(1,1,1,1) * noise (noise.rs:187-211) */
#define RS_TEX_IMAGE   3  /* data = rs_image id; pixel at (u W, (1 - v) H) / 255 (image.rs:34-50) */
typedef struct rs_texture_desc {
    int32_t kind;     /* RS_TEX_SOLID: color = even; RS_TEX_CHECKER: sin(sx)sin(sy)sin(sz) < 0 ? odd : even */
    int32_t data;     /* RS_TEX_PERLIN / RS_TEX_IMAGE: the id returned by rs_perlin / rs_image */
    float   even[4];  /* rgba */
    float   odd[4];   /* rgba */
    double  scale;    /* checker frequency */
} rs_texture_desc;

/* ---- materials (src/material/ *.rs) ---- */
#define RS_MAT_LAMBERTIAN    0
#define RS_MAT_METAL         1
#define RS_MAT_DIFFUSE_METAL 2
#define RS_MAT_DIELECTRIC    3
#define RS_MAT_DIFFUSE_LIGHT 4
#define RS_MAT_MIXED         5
#define RS_MAT_ISOTROPIC     6  /* Isotropic(color = texture.even): SpherePdf (isotropic.rs:25-33) */
#define RS_MAT_BLINN_PHONG   7  /* BlinnPhong(k_specular, exponent, texture): BlinnPhongPdf (blinn_phong.rs:32-42) */
#define RS_NO_MATERIAL      (-1)  /* Option<Arc<dyn Material>> = None */

typedef struct rs_material_desc {
    int32_t kind;
    int32_t glass;            /* Dielectric: 1 = .reflect_curve(Glass{}) (Schlick), 0 = none */
    rs_texture_desc texture;  /* albedo / light texture; Dielectric tint = texture.even */
    double  refractive;       /* Dielectric refractive index */
    double  exponent;         /* DiffuseMetal phong-lobe exponent; BlinnPhong exponent */
    double  multiplier;       /* DiffuseLight multiplier */
    int32_t mix_a, mix_b;     /* MixedMaterial: material ids (already created) */
    double  mix_p;            /* MixedMaterial probability of mix_a */
    double  phong_factor;     /* CommonMaterialSettings.phong_factor (0 = off) */
    int32_t phong_exponent;   /* CommonMaterialSettings.phong_exponent */
    int32_t _pad;
    double  k_specular;       /* BlinnPhong k_specular */
} rs_material_desc;

/* ---- Perlin noise texture data (src/texture/noise.rs) ----
 * The reference builds the tables from a FastRng seeded by the OS (noise.rs:44-66 via
 * FastRng::new()); here the caller passes the tables (include/raysnail.hpp builds them from a
 * seeded FastRng with rand 0.8's shuffle). */
#define RS_PERLIN_NORMAL     0  /* TextureType::Normal: noise(scale p), (n + 1) / 2 for vector values */
#define RS_PERLIN_TURBULENCE 1  /* TextureType::Turbulence(depth) */
#define RS_PERLIN_MARBLE     2  /* TextureType::Marble(depth): (sin(scale z + 10 turb) + 1) / 2 */
#define RS_SMOOTH_NONE       0
#define RS_SMOOTH_LINEAR     1
#define RS_SMOOTH_HERMITE    2
typedef struct rs_perlin_desc {
    uint32_t        point_count;  /* power of two (indices are masked with point_count - 1) */
    int32_t         vector;       /* 1: RandomValueType::Vector (values = 3 doubles each), 0: Float */
    int32_t         smooth;       /* RS_SMOOTH_* */
    int32_t         type;         /* RS_PERLIN_* */
    uint32_t        depth;        /* turbulence / marble depth */
    int32_t         _pad;
    double          scale;
    const double*   values;       /* point_count * (vector ? 3 : 1) */
    const uint32_t* perm_x;       /* point_count each, entries < point_count */
    const uint32_t* perm_y;
    const uint32_t* perm_z;
} rs_perlin_desc;

/* ---- geometry ---- */
#define RS_PLANE_XY 0   /* AARect::new_xy: axes (0,1), fixed 2 */
#define RS_PLANE_XZ 1   /* AARect::new_xz: axes (0,2), fixed 1 */
#define RS_PLANE_YZ 2   /* AARect::new_yz: axes (1,2), fixed 0 */

#define RS_TF_TRANSLATE 0 /* v = offset */
#define RS_TF_ROTATE_X  1 /* v[0] = angle in radians (Transform::rotate_by_x_axis) */
#define RS_TF_ROTATE_Y  2
#define RS_TF_ROTATE_Z  3
#define RS_TF_SCALE     4 /* v = factors */
typedef struct rs_transform {
    int32_t kind;
    int32_t _pad;
    double  v[3];
} rs_transform;

/* ---- camera (CameraBuilder, src/camera.rs:300-413) ---- */
typedef struct rs_camera_desc {
    double   look_from[3];
    double   look_at[3];
    double   vup[3];
    double   fov;        /* vertical field of view, degrees */
    double   aperture;
    double   focus;      /* focus distance */
    double   shutter;    /* shutter speed (ray time = shutter * gen()) */
    uint32_t width, height;
} rs_camera_desc;

/* ---- render settings (TakePhotoSettings src/camera.rs:104-154 + Painter src/painter.rs:69-130) ---- */
#define RS_MODE_AUTO      0
#define RS_MODE_MEGAKERNEL 1  /* one thread per path, all bounces in one launch */
#define RS_MODE_WAVEFRONT  2  /* extend / shade kernels over SoA path queues */
typedef struct rs_render_settings {
    uint32_t samples;    /* requested spp; N = floor(sqrt(samples))^2 is rendered (painter.rs:110-118) */
    uint32_t depth;      /* ray_color recursion depth (default 8, camera.rs:118) */
    int32_t  gamma;      /* 1 = sqrt gamma (into_color, vec3.rs:227-240) */
    int32_t  mode;       /* RS_MODE_* */
    uint64_t seed;       /* frame seed of the determinism contract */
    uint32_t pass;       /* progressive pass index (mixes into the stream key) */
    uint32_t row_begin;  /* rows [row_begin, row_end) with stride row_step are rendered */
    uint32_t row_end;    /* 0 = height */
    uint32_t row_step;   /* 0 or 1 = every row */
} rs_render_settings;

#define RS_KERNEL_NONE       0
#define RS_KERNEL_PATH_MEGA  1  /* k_path_mega: whole path per thread */
#define RS_KERNEL_WF_EXTEND  2  /* k_wf_extend: wavefront traversal (generic scenes) */
#define RS_KERNEL_WFS_EXTEND 3  /* k_wfs_extend: wavefront traversal + material classification */
typedef struct rs_render_stats {
    uint64_t samples;    /* camera samples traced */
    uint64_t segments;   /* world.hit calls (path segments) */
    double   ms;         /* wall time inside the call (device work + sync) */
    double   path_ms;    /* device time of all path-tracing launches (HIP events on the call's stream) */
    uint32_t launches;   /* number of path-tracing launches in the call */
    uint32_t kernel_launches; /* launches of the dominant kernel (megakernel or wavefront extend) */
    double   kernel_ms;  /* device time of those launches (HIP events bracketing each launch) */
    uint64_t kernel_bytes;    /* algorithmic HBM bytes those launches move */
    int32_t  kernel_id;       /* RS_KERNEL_* */
    int32_t  tree_arity;      /* BVH the traversal used: 4 = 4-wide, 2 = binary, 0 = empty world */
} rs_render_stats;

/* What rs_scene_commit built (diagnostic; no reference counterpart: BVH::new_internal,
 * bvh.rs:58-113, builds its own binary tree). */
typedef struct rs_scene_info {
    int32_t  tree_arity;      /* 4: 4-wide tree, near-first traversal; 2: binary tree; 0: empty world */
    int32_t  ref_order;       /* 1: the binary tree is walked in BVH::hit's recursion order (bvh.rs:173-192) */
    int32_t  scene_mode;      /* kernel specialisation: 0 generic, 1 spheres, 2 flat, 3 nest-0, 4 nest-2 */
    int32_t  tree_depth;      /* levels of the tree in use */
    int32_t  stack_need;      /* exact worst-case traversal stack entries of that tree */
    int32_t  stack_lds;       /* entries held in LDS; deeper ones spill to an HBM overflow array */
    uint64_t n_nodes;         /* nodes of the tree in use */
    uint64_t n_objects;       /* object handles (world objects, nested children, lights) */
    uint64_t n_world;         /* objects in the world list (BVH leaves) */
    int32_t  n_devices;       /* devices the scene is committed to */
    uint32_t class_mask;      /* wavefront shading classes some world object's hits fall into (bit k: 0 Lambertian,
                                 1 Metal, 2 DiffuseMetal, 3 Dielectric, 4 generic) */
} rs_scene_info;

typedef struct rs_scene rs_scene;

/* ---- library ---- */
int         rs_abi_version(void);
const char* rs_last_error(void);
int         rs_device_count(int* count);
uint64_t    rs_stream_key(uint64_t seed, uint32_t pass, uint64_t pixel, uint32_t sample);
/* ConstantMedium's Random::normal(): a uniform in [0, 1] from the XorShift128 state (x, y, z, w)
 * at the start of the segment and the medium's handle (see the determinism contract above) */
double      rs_medium_uniform(const uint32_t state[4], uint32_t handle);

/* ---- scene construction ---- */
int rs_scene_create(rs_scene** out);
int rs_scene_destroy(rs_scene* s);
/* texture data referenced by rs_texture_desc.data */
int rs_perlin(rs_scene* s, const rs_perlin_desc* desc, int32_t* id_out);
/* decoded 8-bit RGB pixels, row 0 = top (what DynamicImage::get_pixel indexes, image.rs:34-50) */
int rs_image(rs_scene* s, const uint8_t* rgb, uint32_t width, uint32_t height, int32_t* id_out);
int rs_material(rs_scene* s, const rs_material_desc* desc, int32_t* id_out);
int rs_sphere(rs_scene* s, const double center[3], double radius, const double speed[3] /* NULL = 0 */,
              int32_t material, uint32_t* handle_out);
int rs_aarect(rs_scene* s, int32_t plane, double k, double a0, double a1, double b0, double b1,
              int32_t material, uint32_t* handle_out);
int rs_box(rs_scene* s, const double p0[3], const double p1[3], int32_t material, uint32_t* handle_out);
int rs_quadric(rs_scene* s, const double q[10] /* qa qb qc qd qe qf qg qh qi qj */, int32_t material,
               uint32_t* handle_out);
/* n triangles; pos = n*9 doubles (p0 p1 p2); nrm = n*9 doubles (n0 n1 n2) or NULL (zero normals,
 * Triangle::new default); handles are first_out .. first_out+n-1 */
int rs_triangles(rs_scene* s, const double* pos, const double* nrm, uint32_t n, int32_t material,
                 uint32_t* first_out);
int rs_intersection(rs_scene* s, uint32_t a, uint32_t b, int32_t material, uint32_t* handle_out);
int rs_difference(rs_scene* s, uint32_t plus, uint32_t minus, int32_t material, uint32_t* handle_out);
int rs_transformed(rs_scene* s, uint32_t object, const rs_transform* stack, uint32_t n, uint32_t* handle_out);
/* ConstantMedium::new(boundary, color, density): the medium's material is Isotropic(color) */
int rs_constant_medium(rs_scene* s, uint32_t boundary, const float color[4], double density, uint32_t* handle_out);
int rs_world_add(rs_scene* s, uint32_t handle);
int rs_lights_add(rs_scene* s, uint32_t handle);
int rs_set_background(rs_scene* s, const float lo[3], const float hi[3]);
/* World::new time_limit (world.rs:40-53): bounding boxes of moving spheres span [t0, t1];
 * the reference passes 0..camera.shutter_speed. Default [0, 0]. */
int rs_set_time_range(rs_scene* s, double t0, double t1);
/* freeze the scene: build the BVH and upload it to the current HIP device */
int rs_scene_commit(rs_scene* s);
/* freeze the scene for several devices (Painter::draw's thread fan-out, painter.rs:256-302 and the
 * thread count of :318-325, moved to GPUs): the scene is built once and replicated to each listed
 * HIP device ordinal. A device may be listed more than once (virtual devices with their own streams
 * and buffers). Every rs_render / rs_render_device call then splits its row lattice over the
 * devices the way render_rows interleaves rows over threads (device k of n takes lattice rows
 * k, k+n, ..., painter.rs:248) and runs them concurrently; because every sample owns its RNG
 * stream, the frame is bitwise independent of n. n = 0 is a host-only build: rs_scene_get_info
 * works, rendering returns RS_E_STATE. */
int rs_scene_commit_devices(rs_scene* s, const int* devices, int n);
int rs_scene_get_info(const rs_scene* s, rs_scene_info* out);
/* wavefront lanes for the scene's later renders (1 .. 4; 0 = the defaults): concurrent streams within
 * one frame. The bounce-synchronous wavefront (flat / mesh and rich scenes) deals the chunks of a
 * batch to them round robin (default 2); the streaming wavefront (spheres / box / CSG scenes) deals
 * whole sample batches to lanes, each with its own pool of paths (default 1). No reference
 * counterpart (a scheduling knob like Painter::threads, painter.rs:318-325); frames are bitwise the
 * same. */
int rs_scene_set_lanes(rs_scene* s, uint32_t lanes);
/* frames in flight per device (1 .. 4; default 3): consecutive asynchronous frames are dealt to this
 * many frame slots, each with its own streams and buffers, and a frame waits only for the previous
 * frame of its slot -- the next frame's first paths are traced while the previous frame's last paths
 * drain. Output and stream semantics are unchanged: a frame's result is written on the call's stream,
 * in call order; a frame with a mask (or statistics) also waits for the work queued on its stream
 * before the call. No reference counterpart (painter.rs renders one frame at a time). */
int rs_scene_set_frames_in_flight(rs_scene* s, uint32_t frames);
/* workspace sizes (0 = keep): camera samples per radiance batch buffer (default 32 Mi, whole sample
 * planes are used) and paths per path set (default 256 Mi: the bound of the streaming wavefront's pool
 * -- camera samples injected per iteration times the iterations a path can span; capped per device so
 * that the pools of its frame slots and lanes take at most two thirds of its memory, and, when a frame
 * slot allocates its pool, by the memory then free on the device (other allocations of the process
 * shrink the pool instead of failing the render; RS_E_NOMEM only when not even a 256-path pool fits)
 * -- and the chunk of the bounce-synchronous wavefront). pool_paths is a soft bound: an iteration injects at least 256
 * samples (one block), so a pool below 256 x depth paths is raised to that for the frame.
 * Scheduling only: frames are bitwise the same for any value. */
int rs_scene_set_workspace(rs_scene* s, uint64_t max_batch_items, uint64_t pool_paths);

/* ---- render ---- */
/* host output: out_rgba = W*H*4 floats; mask = W*H bytes or NULL (all pixels) */
int rs_render(rs_scene* s, const rs_camera_desc* cam, const rs_render_settings* st,
              const uint8_t* mask, float* out_rgba, rs_render_stats* stats);
/* host output with progressive row delivery -- Painter::draw's PainterTarget::register_pixels
 * (painter.rs:214) and its end-of-pass sentinel (painter.rs:332). The call's row lattice is rendered
 * in `bands` bands (0 = 16) of consecutive lattice rows, several in flight at once
 * (rs_scene_set_frames_in_flight per device, bands dealt to the devices round robin); as soon as a
 * band is complete, cb(user, y, row, W) is called for each of its rows y (row = out_rgba's row y,
 * already written), from the calling thread, in band order, while the later bands are traced; then
 * cb(user, H, NULL, 0). Rows off the lattice are neither written nor reported. The frame is bitwise
 * the rs_render frame. Stats carry the counts (samples, segments, kernel_bytes, tree_arity) and the call's
 * wall time `ms`; the bands stay in flight together, so no per-kernel device times are taken (0). */
typedef void (*rs_row_callback)(void* user, uint32_t y, const float* row_rgba, uint32_t width);
int rs_render_rows(rs_scene* s, const rs_camera_desc* cam, const rs_render_settings* st, const uint8_t* mask,
                   float* out_rgba, uint32_t bands, rs_row_callback cb, void* user, rs_render_stats* stats);
/* device output: d_out_rgba device pointer (W*H*4 floats), d_mask device pointer or NULL,
 * stream = hipStream_t or NULL (default stream). With stats != NULL the call returns after the
 * work is enqueued AND complete (it synchronises its stream) so that stats are final, and times
 * the dominant kernel's launches; with stats == NULL it returns once the frame is enqueued
 * (asynchronous, no timing events): the frame is complete when `stream` reaches this point, and
 * the next call may be made at once (a call on another stream waits for this frame's buffers).
 * With several devices
 * (rs_scene_commit_devices) d_out_rgba, d_mask and stream belong to the FIRST listed device, which
 * renders its rows in place; the other devices render on their own streams and copy their rows
 * into d_out_rgba at frame end (peer access where the devices allow it). Stats are summed over
 * the devices (kernel_ms / path_ms are device time, ms is the call's wall time). */
int rs_render_device(rs_scene* s, const rs_camera_desc* cam, const rs_render_settings* st,
                     const uint8_t* d_mask, float* d_out_rgba, void* stream, rs_render_stats* stats);
/* n_passes progressive passes of one frame into device frames: pass st->pass + k into d_outs[k] (k < n_passes;
 * the pointers may repeat: later passes overwrite), each frame bitwise the one rs_render_device renders for that
 * pass (no mask: the CLI's pass loop with its never-applied redo map, src/bin/raysnail.rs:379-427). On one device,
 * in the streaming scene modes (spheres, box / CSG: rs_scene_info.scene_mode 1, 3, 4), passes of at most 1 Mi
 * samples -- or 8 Mi at depth >= 16 -- run as sample streams, one per frame slot over a contiguous group of the
 * passes: pass k + 1's camera samples enter the path pool while pass k's paths drain, so the small late launches of
 * a pass carry the next one's work. A stream's path pool bounds the paths its passes can leave in flight: up to
 * depth x one pass's samples per slot, within the caps of rs_scene_set_workspace. Everything else renders the
 * passes one rs_render_device call after the other (larger passes fill the device alone; the stream measured 2-3 %
 * slower there). Stream and stats semantics as rs_render_device (stats summed over the passes). No reference
 * counterpart as one call: the reference renders its passes one after the other (raysnail.rs:379). */
int rs_render_device_passes(rs_scene* s, const rs_camera_desc* cam, const rs_render_settings* st, uint32_t n_passes,
                            float* const* d_outs_rgba, void* stream, rs_render_stats* stats);

/* ---- progressive passes (the CLI's pass loop, src/bin/raysnail.rs:311-427) ----
 * Device-resident frames (RGBA f32, W*H*4), all work on the caller's stream (NULL = default). */
typedef struct rs_noise_stats {
    float    min;        /* min over pixels of calc_noise, starting from 3.0 (raysnail.rs:396) */
    float    max;        /* max, starting from 1.0 (raysnail.rs:397) */
    uint64_t count;      /* pixels with noise >= threshold: the redo map's ones (raysnail.rs:411-422) */
} rs_noise_stats;

/* combine_pixels (raysnail.rs:176-208): acc[i] = new[i] == [0,0,0,0] ? acc[i]
 * : (acc[i] * pass + new[i]) / (pass + 1), per channel in f32. */
int rs_combine_pixels_device(float* d_acc_rgba, const float* d_new_rgba, uint64_t n_pixels, float pass, void* stream);

/* calc_noise (raysnail.rs:150-173) for every pixel -- including upstream's `let x = y` (the 5x5
 * window is centred on column y, the reference colour is pixel (x, y)) -- and the redo map
 * noise >= threshold (raysnail.rs:404-422; the CLI uses 0.01). d_redo may be NULL. Synchronises
 * the stream to return the stats. */
int rs_noise_map_device(const float* d_rgba, uint32_t width, uint32_t height, float threshold, uint8_t* d_redo,
                        void* stream, rs_noise_stats* stats);
/* the same on host buffers (uploaded, computed on the GPU, redo map copied back; redo may be NULL) */
int rs_noise_map(const float* rgba, uint32_t width, uint32_t height, float threshold, uint8_t* redo,
                 rs_noise_stats* stats);

/* ---- diagnostics (parity probes used by tests/) ---- */
/* World::hit (world.rs:63-65) for n rays on the device. rays: n*7 doubles (origin, direction,
 * time); out: n*13 doubles = [hit, t1, t2, p.xyz, n.xyz, u, v, outside, material id] (u, v are
 * computed only in scenes with an Image texture, the only reader: 0 otherwise). The medium key of
 * the probe rays is 0. tmax must be +inf or the hit is dropped when t1 >= tmax. */
int rs_probe_world_hit(rs_scene* s, const double* rays, uint32_t n, double tmin, double tmax, double* out);

/* Radiance of samples s0 .. s0+n-1 of pixel (x, y) -- one ray_color (camera.rs:156-255) each, the
 * camera sample and RNG stream exactly as rs_render draws them (st: samples, depth, seed, pass).
 * out: n*4 doubles = [r, g, b, world.hit count], before the /N and gamma of into_color. Diagnostic
 * (per-sample parity against the oracle); no reference counterpart. */
int rs_probe_samples(rs_scene* s, const rs_camera_desc* cam, const rs_render_settings* st, uint32_t x, uint32_t y,
                     uint32_t s0, uint32_t n, double* out);

#ifdef __cplusplus
}
#endif
#endif /* RAYSNAIL_HIP_H */
