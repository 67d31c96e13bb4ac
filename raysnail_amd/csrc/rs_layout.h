// rs_layout.h — device-resident scene layout (host builds it, kernels read it).
//
// Everything is f64, the reference's arithmetic type (src/prelude/vec3.rs:14-19); colours stay
// f32 like the reference's Color (src/prelude/color.rs:11-16). The scene for every config fits
// in a few MB, so it is L2/MALL-resident during a frame; per-path state is what streams.
#pragma once
#include <stdint.h>

#define RS_MAX_NEST 4   // object nesting levels supported on the GPU (TfFacade / CSG chains)

namespace rs {

enum PrimKind : int32_t {
    PK_SPHERE = 0,
    PK_RECT = 1,
    PK_BOX = 2,
    PK_QUADRIC = 3,
    PK_TRIANGLE = 4,
    PK_AND = 5,     // csg Intersection  (src/hittable/csg/intersection.rs)
    PK_SUB = 6,     // csg Difference    (src/hittable/csg/difference.rs)
    PK_XFORM = 7,   // TfFacade          (src/hittable/transform/tf_facade.rs)
    PK_MEDIUM = 8,  // ConstantMedium    (src/hittable/medium/constant.rs)
};

// One entry per hittable handle (world objects and nested children alike).
struct DPrim {
    int32_t kind;
    int32_t idx;   // index into the per-kind array
    int32_t mat;   // material id, -1 = None
    int32_t aux;   // XFORM: number of transforms; CSG: unused
};

struct DSphere {   // sphere.rs:16-23
    double c[3];
    double r;
    double r2;     // radius_squared
    double v[3];   // speed
};

// A static sphere in 32 bytes (spheres-only scenes without motion: the traversal's leaf record):
// radius_squared is radius * radius (sphere.rs:35-43), recomputed by the same f64 multiply.
struct alignas(32) DSphereS {
    double c[3];
    double r;
};

struct DRect {     // rect.rs:178-212
    int32_t ax0, ax1, ax2, pad;
    double k, a0, a1, b0, b1;
};

struct DBox {      // box.rs:331-336 (faces are derived from min/max in the reference order)
    double mn[3];
    double mx[3];
};

struct DQuadric {  // quadric.rs:20-34, field order qa qb qc qd qe qf qg qh qi qj
    double q[10];
};

struct DTri {      // triangle_mesh.rs:14-26
    double p0[3];
    double a, b, c, d, e, f;
    double n0[3], n1[3], n2[3];
};

struct DCsg {      // Intersection(o1, o2) / Difference(plus, minus): prim indices
    int32_t a, b;
};

struct DMedium {   // ConstantMedium(boundary, Isotropic(color), density): constant.rs:13-39
    int32_t boundary;        // prim index of the boundary object
    int32_t mat;             // the Isotropic material created for it
    double neg_inv_density;  // -1 / density
};

struct DXform {    // TfFacade: child prim + transforms [first, first+n) of the matrix table
    int32_t child;
    int32_t first;
};

// rows 0..2 of the 4x4 row-major matrix (row 3 is never read by row_mat4_transform's xyz)
struct DMat34 {
    double m[3][4];
};

struct DMaterial { // src/material/*.rs flattened
    int32_t kind;        // RS_MAT_*
    int32_t tex_kind;    // RS_TEX_*
    int32_t tex_data;    // RS_TEX_PERLIN: DPerlin index; RS_TEX_IMAGE: DImage index
    int32_t pad0;
    int32_t glass;
    int32_t mix_a, mix_b;
    int32_t phong_exponent;  // effective settings() (MixedMaterial -> material_1's)
    float even[4];
    float odd[4];
    double tex_scale;
    double enter_refractive, outer_refractive;
    double exponent;
    double multiplier;
    double mix_p;
    double phong_factor;
    double k_specular;   // BlinnPhong
};

struct DPerlin {   // noise.rs:28-37 (tables in DScene::tex_f64 / tex_i32)
    int32_t point_count, vector, smooth, type;
    int32_t depth;
    int32_t voff;        // values: tex_f64[voff ..], 3 per point (vector) or 1
    int32_t poff;        // perm_x, perm_y, perm_z: tex_i32[poff ..], point_count each
    int32_t pad;
    double scale;
};

struct DImage {    // image.rs: 8-bit RGB, row 0 = top, at DScene::tex_u8[off ..]
    uint32_t w, h;
    uint64_t off;
};

// Binary BVH node: both child boxes live in the parent, so one 64-byte fetch tests two children.
// child >= 0: inner node index; INT32_MIN: empty slot; other child < 0: a leaf. In flat scenes
// (meshes) the leaf holds leaf entry ~child: entries are in tree order (the leaves of a node are
// adjacent in memory), DScene::lprim maps an entry to its prim handle and ltri holds what the leaf
// test reads; in the other scenes ~child is the prim handle itself (lprim null).
// Boxes are f32 rounded OUTWARD: inner-node tests only cull (conservatively); every leaf is
// re-tested against the object's exact f64 bbox (DScene::pbox) before the object itself, which
// is what BVH::hit does with the leaf's own box (bvh.rs:173-177).
struct alignas(64) DNode {
    float lo[2][3];
    float hi[2][3];
    int32_t child[2];
    int32_t pad[2];
};

// 4-wide node (monotone scenes, near-first traversal): SoA child boxes (f32, rounded outward) so one
// 128-byte fetch tests four children; child codes as in DNode.
struct alignas(128) DNode4 {
    float lo_x[4], lo_y[4], lo_z[4];
    float hi_x[4], hi_y[4], hi_z[4];
    int32_t child[4];
    int32_t pad[4];
};

// Triangle data in BVH leaf order (flat scenes): what Triangle::hit's accept test reads
// (triangle_mesh.rs:85-131: p0 and the edges a..f), so a leaf's triangles are contiguous and the
// traversal needs no DPrim hop; the winner's full record (normals) is rebuilt from DTri.
struct alignas(16) LTri {
    double p0[3];
    double a, b, c, d, e, f;
    double kind;   // PrimKind of the entry as a double (only PK_TRIANGLE entries carry the fields above)
};

struct DBox64 {    // an object's reference bbox (exact f64), tested before its hit()
    double lo[3];
    double hi[3];
};

// tables of the LDS image (DScene::limg_off), in image order
enum LimgTable { LT_NODES4 = 0, LT_PBOX, LT_PCLASS, LT_PRIMS, LT_SPHERES, LT_RECTS, LT_BOXES, LT_QUADRICS, LT_CSGS,
                 LT_XFORMS, LT_TF_FWD, LT_TF_INV, LT_COUNT };
// LDS bytes the image may take: the nest-mode extend keeps 4 blocks of 256 per CU, each with its
// 16-entry traversal stack (stack_lds: 16 KiB) and the image, 4 x (16 + 15) KiB = 124 KiB <= 160 KiB
// (rs_internal.h checks it against the CU's LDS)
constexpr uint32_t kLimgMax = 15u * 1024u;

struct DScene {
    const DNode* nodes;      // binary tree (reference-order scenes)
    const DNode4* nodes4;    // 4-wide tree (monotone scenes), root = root4
    const DBox64* pbox;      // per prim handle
    const uint8_t* pclass;   // per prim handle: wavefront shading class of its material (spheres-only scenes)
    const DPrim* prims;
    const DSphere* spheres;
    const int32_t* lprim;    // leaf entry -> prim handle (flat scenes; null: leaf codes are ~prim)
    const DSphere* lsph;     // spheres-only scenes: the sphere of prim handle p at lsph[p] (no DPrim hop)
    const DSphereS* lsphs;   // the same in 32-byte records when no sphere moves (twice the records per cache line)
    const LTri* ltri;        // flat scenes: the triangle of each leaf entry (+ every entry's kind)
    const DRect* rects;
    const DBox* boxes;
    const DQuadric* quadrics;
    const DTri* tris;
    const DCsg* csgs;
    const DXform* xforms;
    const DMat34* tf_fwd;
    const DMat34* tf_inv;
    const DMaterial* mats;
    const DMedium* media;
    const DPerlin* perlins;
    const DImage* images;
    const double* tex_f64;
    const int32_t* tex_i32;
    const uint8_t* tex_u8;
    const int32_t* lights;   // prim indices
    // Traversal-stack overflow: entries [kStackMax, stack_need) of a thread's stack live in HBM,
    // column (blockIdx.x * kBlock + threadIdx.x) of a [stack_need - kStackMax][gridDim.x * kBlock]
    // array that the host sizes per launch grid (null when the tree fits the LDS stack).
    int32_t* stk_ovf;
    // Nest modes: the small tables a traversal reads (4-wide tree, own boxes, classes, object records)
    // as one image that the extend's blocks copy into LDS (rs_kernels.hip lds_scene), so the dependent
    // node -> prim -> CSG -> child -> shape loads of a nested-object test are LDS reads. Null (and
    // limg_bytes 0) when the scene's tables exceed kLimgMax.
    const void* limg;
    uint32_t limg_bytes;                  // a multiple of 16
    uint32_t limg_off[LT_COUNT];          // byte offset of each table in the image (LimgTable order)
    int32_t n_lights;
    int32_t root;            // root child code (node index, or ~prim if a single object, or INT32_MIN if empty)
    int32_t default_mat;     // world.rs:51 Lambertian(Color(1,1,1,1))
    int32_t ref_order;       // 1: traverse in BVH::hit's recursion order (bvh.rs:173-192); 0: near-first
    int32_t root4;           // root of nodes4 (>= 0) when the 4-wide tree is used, else -1
    int32_t uv;              // 1: hit records carry (u, v) (some texture reads them: Image)
    int32_t has_media;       // 1: the scene has ConstantMedium objects (rays carry the medium key)
    int32_t stack_need;      // exact worst-case traversal stack depth of the tree in use (host-computed)
    int32_t moving;          // 1: some sphere has a nonzero speed (center_at needs the time)
    int32_t ltop;            // spheres mode: the first ltop nodes of nodes4 (breadth-first, root 0) are the tree's
                             // top, which the extend's blocks also hold in LDS (rs_kernels.hip s_top4); 0: none
    int32_t lamb_only;       // 1: every prim's hits carry a Lambertian or a DiffuseLight material (shading classes
                             // 0 and 6 only): the flat scenes' shading kernel compiled for Lambertian alone
    float bg_lo[4], bg_hi[4];
};

// nodes of the spheres mode's tree top held in LDS per extend block: the root and three levels (85 nodes, 10.6 KiB;
// with the 16-entry stack 27 KiB per block, 5 blocks per CU). Bench frame: none 7.08 ms, 21 nodes 6.94, 85 nodes
// 6.86 (profiles/r5/ab/variants_ltop_r5e.txt)
#ifndef RS_LTOP
#define RS_LTOP 85
#endif
constexpr int kLTop = RS_LTOP;


struct DCamera {   // camera.rs:18-31
    double origin[3], lb[3], hf[3], vf[3], hu[3], vu[3];
    double aperture, shutter;
};

}  // namespace rs
