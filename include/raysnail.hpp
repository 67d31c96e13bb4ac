/*
 * raysnail.hpp -- C++ host API for the GPU render path (libraysnail_host.so over libraysnail_hip.so).
 *
 * raysnail's own host side is Rust and there is no Rust toolchain in this build, so this header is
 * the compiled host layer above the C-ABI (include/raysnail_hip.h). It keeps the reference's
 * names and argument meaning so code written against raysnail reads the same:
 *
 *   auto cam   = CameraBuilder().look_from({13, 2, 3}).look_at({0, 0, 0}).fov(20).aperture(0.02)
 *                    .focus(10).width(800).height(500).build();              // src/camera.rs:300-413
 *   World world(hittables, lights, Gradient{}, {0.0, cam.shutter_speed()});  // src/hittable/collection/world.rs
 *   auto pixels = cam.take_photo().samples(64).depth(8).shot(nullptr, world);   // src/camera.rs:261-295
 *
 * and the SDL front end (src/sdl_parser.rs) with the CLI's scene conventions (src/bin/raysnail.rs:340-373):
 *
 *   SceneData sd = SdlParser::parse("scene.sdl");
 *   CliScene  sc = cli_scene(std::move(sd), 800, 500);
 *
 * Objects are shared_ptr graphs (the reference's Arc<dyn ...>). A World is exported once into a
 * scene sink -- libraysnail_hip (rs_*), or any table with the same signatures (the tests replay
 * the identical call sequence into the CPU oracle) -- with shared objects exported once.
 * Errors: the reference panics (aborts); here every failure throws raysnail::Error.
 */
#pragma once

#include <array>
#include <cstdint>
#include <functional>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "raysnail_hip.h"

namespace raysnail {

class Error : public std::runtime_error {
public:
    Error(int code, const std::string& msg) : std::runtime_error(msg), code_(code) {}
    int code() const { return code_; }
private:
    int code_;
};

// ---------------------------------------------------------------------------------- prelude ----
struct Vec3 {  // src/prelude/vec3.rs (only what the host side needs)
    double x = 0.0, y = 0.0, z = 0.0;
};
using Point3 = Vec3;

struct Color {  // src/prelude/color.rs:11-47 (f32 rgba)
    float r = 0.f, g = 0.f, b = 0.f, a = 1.f;
    static Color new64(double r, double g, double b, double a) {
        return Color{(float)r, (float)g, (float)b, (float)a};
    }
};

// -------------------------------------------------------------------------------- FastRng ----
// src/prelude/random.rs:109-145: XorShiftRng (rand_xorshift 0.3.0) seeded by rand_core 0.6's
// seed_from_u64. The reference seeds it from the OS (FastRng::new); here the seed is explicit.
class FastRng {
public:
    explicit FastRng(uint64_t seed);
    uint32_t next_u32();
    uint64_t next_u64();
    double gen();                          // next_u64 as f64 / u64::MAX as f64, in [0, 1]
    double range(double start, double end) { return start + gen() * (end - start); }
    // rand 0.8.3 SliceRandom::shuffle: for i in (1..len).rev() swap(i, gen_range(0..i+1)), with
    // UniformInt<u32>::sample_single's widening-multiply rejection (third-party, restated)
    void shuffle(std::vector<uint32_t>& v);
    uint32_t gen_index(uint32_t ubound);
private:
    uint32_t x_, y_, z_, w_;
};

// ---------------------------------------------------------------------------------- textures ----
enum class SmoothType { None = RS_SMOOTH_NONE, LinearInterpolate = RS_SMOOTH_LINEAR, HermitianCubic = RS_SMOOTH_HERMITE };

struct PerlinData {  // the tables of texture/noise.rs:28-37 + the texture settings
    uint32_t point_count = 0;
    bool vector = false;
    SmoothType smooth = SmoothType::HermitianCubic;
    int32_t type = RS_PERLIN_NORMAL;
    uint32_t depth = 0;
    double scale = 1.0;
    std::vector<double> values;                    // 3 per point (Vector) or 1 (Float)
    std::vector<uint32_t> perm_x, perm_y, perm_z;
};

class Perlin {  // src/texture/noise.rs
public:
    // Perlin::new (noise.rs:44-66): values Vec3::random_unit / gen, then three shuffled permutations
    Perlin(size_t point_count, bool vector, FastRng& rng);
    Perlin& scale(double s) { d_->scale = s; return *this; }
    Perlin& smooth(SmoothType t) { d_->smooth = t; return *this; }
    Perlin& turbulence(uint8_t depth) { d_->type = RS_PERLIN_TURBULENCE; d_->depth = depth; return *this; }
    Perlin& marble(uint8_t depth) { d_->type = RS_PERLIN_MARBLE; d_->depth = depth; return *this; }
    const std::shared_ptr<PerlinData>& data() const { return d_; }
private:
    std::shared_ptr<PerlinData> d_;
};

struct ImageData {  // decoded 8-bit RGB, row 0 = top
    uint32_t width = 0, height = 0;
    std::vector<uint8_t> rgb;
};

class Image {  // src/texture/image.rs
public:
    // Image::new (image.rs:24-31): decodes a PNG (8-bit gray / gray-alpha / RGB / RGBA / palette,
    // non-interlaced); throws Error like the reference's Err(String)
    static Image open(const std::string& path);
    Image(uint32_t width, uint32_t height, std::vector<uint8_t> rgb);
    const std::shared_ptr<const ImageData>& data() const { return d_; }
private:
    std::shared_ptr<const ImageData> d_;
};

// Arc<dyn Texture>: a solid Color (color.rs:61-65), a Checker (texture/checker.rs:13-30), a Perlin
// noise (texture/noise.rs) or an Image (texture/image.rs).
struct Texture {
    int32_t kind = RS_TEX_SOLID;
    Color odd, even;
    double scale = 1.0;
    std::shared_ptr<const PerlinData> perlin;
    std::shared_ptr<const ImageData> image;
    static Texture color(const Color& c) { Texture t; t.kind = RS_TEX_SOLID; t.odd = t.even = c; return t; }
    static Texture checker(const Color& odd, const Color& even, double scale) {
        Texture t; t.kind = RS_TEX_CHECKER; t.odd = odd; t.even = even; t.scale = scale; return t;
    }
    static Texture noise(const Perlin& p) {
        Texture t; t.kind = RS_TEX_PERLIN; t.perlin = std::make_shared<const PerlinData>(*p.data()); return t;
    }
    static Texture of(const Image& i) { Texture t; t.kind = RS_TEX_IMAGE; t.image = i.data(); return t; }
};

class SceneSink;

// --------------------------------------------------------------------------------- materials ----
struct CommonMaterialSettings {  // src/material/mod.rs:41-54
    double phong_factor = 0.0;
    int32_t phong_exponent = 1;
};

class Material {
public:
    virtual ~Material() = default;
    virtual int32_t export_to(SceneSink& sink) const = 0;
    virtual CommonMaterialSettings settings() const { return settings_; }
    void set(const CommonMaterialSettings& s) { settings_ = s; }
protected:
    rs_material_desc base_desc(SceneSink& sink, int32_t kind, const Texture& t) const;
    CommonMaterialSettings settings_;
};
using MaterialRef = std::shared_ptr<const Material>;

class Lambertian : public Material {  // src/material/lambertian.rs
public:
    explicit Lambertian(Texture t) : tex_(t) {}
    int32_t export_to(SceneSink& sink) const override;
private:
    Texture tex_;
};

class Metal : public Material {  // src/material/metal.rs:86-118
public:
    explicit Metal(Texture t) : tex_(t) {}
    int32_t export_to(SceneSink& sink) const override;
private:
    Texture tex_;
};

class DiffuseMetal : public Material {  // src/material/metal.rs:36-68
public:
    DiffuseMetal(double exponent, Texture t) : exponent_(exponent), tex_(t) {}
    int32_t export_to(SceneSink& sink) const override;
private:
    double exponent_;
    Texture tex_;
};

struct Glass {};  // src/material/dielectric.rs:17-25 (the only ReflectCurve upstream)

class Dielectric : public Material {  // src/material/dielectric.rs:27-93
public:
    Dielectric(Color color, double refractive) : color_(color), refractive_(refractive) {}
    Dielectric& reflect_curve(Glass) { glass_ = true; return *this; }
    int32_t export_to(SceneSink& sink) const override;
private:
    Color color_;
    double refractive_;
    bool glass_ = false;
};

class DiffuseLight : public Material {  // src/material/light.rs
public:
    explicit DiffuseLight(Texture t) : tex_(t) {}
    DiffuseLight& multiplier(double m) { mult_ = m; return *this; }
    int32_t export_to(SceneSink& sink) const override;
private:
    Texture tex_;
    double mult_ = 1.0;
};

class Isotropic : public Material {  // src/material/isotropic.rs
public:
    explicit Isotropic(Color c) : color_(c) {}
    int32_t export_to(SceneSink& sink) const override;
private:
    Color color_;
};

class BlinnPhong : public Material {  // src/material/blinn_phong.rs
public:
    BlinnPhong(double k_specular, double exponent, Texture t) : k_(k_specular), e_(exponent), tex_(t) {}
    int32_t export_to(SceneSink& sink) const override;
private:
    double k_, e_;
    Texture tex_;
};

class MixedMaterial : public Material {  // src/material/mixed_material.rs
public:
    MixedMaterial(MaterialRef m1, MaterialRef m2, double probability_1)
        : m1_(std::move(m1)), m2_(std::move(m2)), p_(probability_1) {}
    int32_t export_to(SceneSink& sink) const override;
    CommonMaterialSettings settings() const override { return m1_->settings(); }
private:
    MaterialRef m1_, m2_;
    double p_;
};

// ---------------------------------------------------------------------------------- geometry ----
class Hittable {
public:
    virtual ~Hittable() = default;
    // handles of this object in the sink (a mesh is one handle per triangle)
    virtual std::vector<uint32_t> export_to(SceneSink& sink) const = 0;
};
using HittableRef = std::shared_ptr<const Hittable>;

class Sphere : public Hittable {  // src/hittable/geometry/sphere.rs
public:
    Sphere(Point3 center, double radius, MaterialRef material)
        : c_(center), r_(radius), mat_(std::move(material)) {}
    Sphere& with_speed(Vec3 speed) { speed_ = speed; return *this; }
    std::vector<uint32_t> export_to(SceneSink& sink) const override;
private:
    Point3 c_;
    double r_;
    Vec3 speed_;
    MaterialRef mat_;
};

struct AARectMetrics {  // src/hittable/geometry/rect.rs:17-37 (requires a0 < a1 and b0 < b1)
    double k;
    std::pair<double, double> a, b;
    AARectMetrics(double k, std::pair<double, double> a, std::pair<double, double> b);
};

class AARect : public Hittable {  // src/hittable/geometry/rect.rs
public:
    static std::shared_ptr<AARect> new_xy(AARectMetrics m, MaterialRef mat) { return std::make_shared<AARect>(RS_PLANE_XY, m, mat); }
    static std::shared_ptr<AARect> new_xz(AARectMetrics m, MaterialRef mat) { return std::make_shared<AARect>(RS_PLANE_XZ, m, mat); }
    static std::shared_ptr<AARect> new_yz(AARectMetrics m, MaterialRef mat) { return std::make_shared<AARect>(RS_PLANE_YZ, m, mat); }
    AARect(int32_t plane, AARectMetrics m, MaterialRef mat) : plane_(plane), m_(m), mat_(std::move(mat)) {}
    std::vector<uint32_t> export_to(SceneSink& sink) const override;
private:
    int32_t plane_;
    AARectMetrics m_;
    MaterialRef mat_;
};

class Box : public Hittable {  // src/hittable/geometry/box.rs
public:
    Box(Point3 p0, Point3 p1, MaterialRef mat) : p0_(p0), p1_(p1), mat_(std::move(mat)) {}
    std::vector<uint32_t> export_to(SceneSink& sink) const override;
private:
    Point3 p0_, p1_;
    MaterialRef mat_;
};

class Quadric : public Hittable {  // src/hittable/geometry/quadric.rs (field order qa..qj)
public:
    Quadric(double qa, double qb, double qc, double qd, double qe, double qf, double qg, double qh, double qi,
            double qj, MaterialRef mat)
        : q_{qa, qb, qc, qd, qe, qf, qg, qh, qi, qj}, mat_(std::move(mat)) {}
    std::vector<uint32_t> export_to(SceneSink& sink) const override;
private:
    std::array<double, 10> q_;
    MaterialRef mat_;
};

class TriangleMesh : public Hittable {  // src/hittable/geometry/triangle_mesh.rs (one Triangle per face)
public:
    // positions: 9 doubles per triangle; normals: 9 per triangle or empty (zero normals)
    TriangleMesh(std::vector<double> positions, std::vector<double> normals, MaterialRef mat);
    // TriangleMesh::load (triangle_mesh.rs:166-276): an OBJ file through a tobj-4.0.2-compatible
    // reader (single_index, triangulate), each vertex rotated about `axis` by rotation_angle degrees,
    // then p * scale + offset; vertex normals from the file (rotated) or the averaged unit face
    // normals of the rotated positions
    static std::shared_ptr<TriangleMesh> load(const std::string& filename, double scale, Vec3 offset,
                                              double rotation_angle, int axis, MaterialRef material);
    size_t len() const { return pos_.size() / 9; }
    const std::vector<double>& positions() const { return pos_; }
    const std::vector<double>& normals() const { return nrm_; }
    std::vector<uint32_t> export_to(SceneSink& sink) const override;
private:
    std::vector<double> pos_, nrm_;
    MaterialRef mat_;
};

class Intersection : public Hittable {  // src/hittable/csg/intersection.rs
public:
    Intersection(HittableRef o1, HittableRef o2, MaterialRef mat)
        : o1_(std::move(o1)), o2_(std::move(o2)), mat_(std::move(mat)) {}
    std::vector<uint32_t> export_to(SceneSink& sink) const override;
private:
    HittableRef o1_, o2_;
    MaterialRef mat_;
};

class Difference : public Hittable {  // src/hittable/csg/difference.rs
public:
    Difference(HittableRef plus, HittableRef minus, MaterialRef mat)
        : plus_(std::move(plus)), minus_(std::move(minus)), mat_(std::move(mat)) {}
    std::vector<uint32_t> export_to(SceneSink& sink) const override;
private:
    HittableRef plus_, minus_;
    MaterialRef mat_;
};

struct Transform {  // src/hittable/transform/transform.rs:16-107 (angles in radians)
    rs_transform t;
    static Transform translate(Vec3 v) { return make(RS_TF_TRANSLATE, v); }
    static Transform rotate_by_x_axis(double theta) { return make(RS_TF_ROTATE_X, {theta, 0, 0}); }
    static Transform rotate_by_y_axis(double theta) { return make(RS_TF_ROTATE_Y, {theta, 0, 0}); }
    static Transform rotate_by_z_axis(double theta) { return make(RS_TF_ROTATE_Z, {theta, 0, 0}); }
    static Transform scale(Vec3 v) { return make(RS_TF_SCALE, v); }
private:
    static Transform make(int32_t kind, Vec3 v) {
        Transform x{};
        x.t.kind = kind; x.t.v[0] = v.x; x.t.v[1] = v.y; x.t.v[2] = v.z;
        return x;
    }
};

class TransformStack {  // src/hittable/transform/transform.rs:110-157
public:
    void push(const Transform& t) { stack_.push_back(t.t); }
    size_t len() const { return stack_.size(); }
    const std::vector<rs_transform>& items() const { return stack_; }
private:
    std::vector<rs_transform> stack_;
};

class ConstantMedium : public Hittable {  // src/hittable/medium/constant.rs (material Isotropic(color))
public:
    ConstantMedium(HittableRef boundary, Color color, double density)
        : boundary_(std::move(boundary)), color_(color), density_(density) {}
    std::vector<uint32_t> export_to(SceneSink& sink) const override;
private:
    HittableRef boundary_;
    Color color_;
    double density_;
};

class HittableList;

// A BVH (or HittableList) used as one object of another list (bvh.rs, list.rs). The device scene
// has one BVH over every object, so a group exports its members; a TfFacade of a group becomes a
// TfFacade of each member (the same closest hit for spheres / rects / triangles; for
// order-dependent members the group's own BVH order is not kept).
class BVH : public Hittable {
public:
    BVH(const HittableList& list, std::pair<double, double> time_limit = {0.0, 0.0});
    std::vector<uint32_t> export_to(SceneSink& sink) const override;
private:
    std::vector<HittableRef> objects_;
};

class TfFacade : public Hittable {  // src/hittable/transform/tf_facade.rs
public:
    TfFacade(HittableRef obj, TransformStack stack) : obj_(std::move(obj)), stack_(std::move(stack)) {}
    std::vector<uint32_t> export_to(SceneSink& sink) const override;
private:
    HittableRef obj_;
    TransformStack stack_;
};

class HittableList {  // src/hittable/collection/list.rs
public:
    HittableList& add(HittableRef o) { objects_.push_back(std::move(o)); return *this; }
    size_t len() const { return objects_.size(); }
    const std::vector<HittableRef>& objects() const { return objects_; }
private:
    std::vector<HittableRef> objects_;
};

// The background closure of every reference front end: lo.gradient(hi, (d.y + 1) / 2)
// (examples/rtow_13_1.rs:38-41, src/bin/raysnail.rs:364-367, src/prelude/color.rs:50-58).
struct Gradient {
    Color lo{0.3f, 0.4f, 0.5f, 1.f};
    Color hi{0.7f, 0.89f, 1.0f, 1.f};
};

// ------------------------------------------------------------------------------ scene sinks ----
// The scene-building half of the C-ABI as a table, so one export routine feeds libraysnail_hip or
// any backend with identical signatures (the CPU oracle in the tests).
extern "C" {
typedef struct rsh_sink_api {
    int (*material)(void* s, const rs_material_desc* d, int32_t* id);
    int (*sphere)(void* s, const double* c, double r, const double* speed, int32_t mat, uint32_t* h);
    int (*aarect)(void* s, int32_t plane, double k, double a0, double a1, double b0, double b1, int32_t mat, uint32_t* h);
    int (*box)(void* s, const double* p0, const double* p1, int32_t mat, uint32_t* h);
    int (*quadric)(void* s, const double* q, int32_t mat, uint32_t* h);
    int (*triangles)(void* s, const double* pos, const double* nrm, uint32_t n, int32_t mat, uint32_t* first);
    int (*intersection)(void* s, uint32_t a, uint32_t b, int32_t mat, uint32_t* h);
    int (*difference)(void* s, uint32_t a, uint32_t b, int32_t mat, uint32_t* h);
    int (*transformed)(void* s, uint32_t obj, const rs_transform* st, uint32_t n, uint32_t* h);
    int (*world_add)(void* s, uint32_t h);
    int (*lights_add)(void* s, uint32_t h);
    int (*set_background)(void* s, const float* lo, const float* hi);
    int (*set_time_range)(void* s, double t0, double t1);
    int (*perlin)(void* s, const rs_perlin_desc* d, int32_t* id);
    int (*image)(void* s, const uint8_t* rgb, uint32_t w, uint32_t h, int32_t* id);
    int (*constant_medium)(void* s, uint32_t boundary, const float* color, double density, uint32_t* h);
    const char* (*last_error)(void);
} rsh_sink_api;
}

const rsh_sink_api& hip_sink_api();  // libraysnail_hip's rs_* functions

class SceneSink {
public:
    SceneSink(const rsh_sink_api& api, void* scene) : api(api), scene(scene) {}
    void check(int rc) const;
    const rsh_sink_api& api;
    void* scene;
    std::unordered_map<const void*, int32_t> materials;              // exported once each
    std::unordered_map<const void*, int32_t> textures;               // Perlin / Image data, once each
    int32_t texture_data(const Texture& t);
    std::unordered_map<const void*, std::vector<uint32_t>> objects;
    int32_t material(const MaterialRef& m);
    std::vector<uint32_t> object(const HittableRef& o);
};

// -------------------------------------------------------------------------------------- World ----
class World {  // src/hittable/collection/world.rs:20-79
public:
    World(HittableList hittables, HittableList lights, Gradient background = Gradient{},
          std::pair<double, double> time_range = {0.0, 0.0});
    ~World();
    World(World&&) noexcept;
    World& operator=(World&&) noexcept;
    World(const World&) = delete;
    World& operator=(const World&) = delete;

    void export_to(SceneSink& sink) const;   // background, time range, world list, lights list
    rs_scene* device_scene();                // exported + committed on first use (BVH build + upload)
    const HittableList& hittables() const { return hittables_; }
    const HittableList& lights() const { return lights_; }
private:
    HittableList hittables_, lights_;
    Gradient background_;
    std::pair<double, double> time_range_;
    rs_scene* scene_ = nullptr;
};

// ------------------------------------------------------------------------------------- Camera ----
class TakePhotoSettings;

class Camera {  // src/camera.rs:18-91 (the basis is computed inside the library, camera.rs:37-73)
public:
    explicit Camera(const rs_camera_desc& d) : desc_(d) {}
    const rs_camera_desc& desc() const { return desc_; }
    double shutter_speed() const { return desc_.shutter; }
    size_t picture_width() const { return desc_.width; }
    size_t picture_height() const { return desc_.height; }
    TakePhotoSettings take_photo() const;
private:
    rs_camera_desc desc_;
};

class CameraBuilder {  // src/camera.rs:300-413 (defaults :314-329)
public:
    CameraBuilder();
    CameraBuilder& look_from(Point3 p) { d_.look_from[0] = p.x; d_.look_from[1] = p.y; d_.look_from[2] = p.z; return *this; }
    CameraBuilder& look_at(Point3 p) { d_.look_at[0] = p.x; d_.look_at[1] = p.y; d_.look_at[2] = p.z; return *this; }
    CameraBuilder& vup(Vec3 v) { d_.vup[0] = v.x; d_.vup[1] = v.y; d_.vup[2] = v.z; return *this; }
    CameraBuilder& fov(double f) { d_.fov = f; return *this; }
    CameraBuilder& aperture(double a) { d_.aperture = a; return *this; }
    CameraBuilder& focus(double f) { d_.focus = f; return *this; }
    CameraBuilder& focus_to_look_at();
    CameraBuilder& shutter_speed(double s) { d_.shutter = s; return *this; }
    CameraBuilder& width(size_t w) { d_.width = (uint32_t)w; return *this; }
    CameraBuilder& height(size_t h) { d_.height = (uint32_t)h; return *this; }
    Camera build() const { return Camera(d_); }
private:
    rs_camera_desc d_;
};

// ------------------------------------------------------------------------------------ Painter ----
using Pixel = std::array<float, 4>;

struct PainterTarget {  // src/painter.rs:23-27
    virtual ~PainterTarget() = default;
    virtual void register_pixels(size_t y, const std::vector<Pixel>& pixels) = 0;
};
struct PainterController {  // src/painter.rs:28-32 (never polled upstream)
    virtual ~PainterController() = default;
};
struct PixelController {  // src/painter.rs:34-38
    virtual ~PixelController() = default;
    virtual bool calculate_pixel(size_t x, size_t y) const = 0;
};

class TakePhotoSettings {  // src/camera.rs:103-154 + the GPU painter knobs (seed / pass / rows / mode)
public:
    explicit TakePhotoSettings(const Camera& c) : camera_(c) {}
    TakePhotoSettings& depth(size_t d) { depth_ = (uint32_t)d; return *this; }
    TakePhotoSettings& gamma(bool g) { gamma_ = g; return *this; }
    TakePhotoSettings& samples(size_t s) { samples_ = (uint32_t)s; return *this; }
    TakePhotoSettings& threads(size_t) { return *this; }   // CPU painter knobs: no meaning on the GPU
    TakePhotoSettings& parallel(bool) { return *this; }
    TakePhotoSettings& seed(uint64_t s) { seed_ = s; return *this; }
    TakePhotoSettings& pass_index(uint32_t p) { pass_ = p; return *this; }
    TakePhotoSettings& rows(uint32_t begin, uint32_t end = 0, uint32_t step = 1) {
        row_begin_ = begin; row_end_ = end; row_step_ = step; return *this;
    }
    TakePhotoSettings& mode(int32_t m) { mode_ = m; return *this; }
    rs_render_settings settings() const;

    // src/camera.rs:261-287: rows go to target (then the (height, []) sentinel, painter.rs:332)
    std::vector<Pixel> shot_to_target(const char* path, World& world, PainterTarget* target,
                                      PainterController* controller, const PixelController* pixel_map);
    std::vector<Pixel> shot(const char* path, World& world) { return shot_to_target(path, world, nullptr, nullptr, nullptr); }
    const rs_render_stats& last_stats() const { return stats_; }
private:
    Camera camera_;
    uint32_t depth_ = 8, samples_ = 50, pass_ = 0, row_begin_ = 0, row_end_ = 0, row_step_ = 1;
    bool gamma_ = true;
    uint64_t seed_ = 0;
    int32_t mode_ = RS_MODE_AUTO;
    rs_render_stats stats_{};
};

inline TakePhotoSettings Camera::take_photo() const { return TakePhotoSettings(*this); }

// src/bin/raysnail.rs:176-208 combine_pixel: keep old where new is [0,0,0,0], else (old p + new)/(p + 1)
void combine_pixels(std::vector<Pixel>& old_pixels, const std::vector<Pixel>& new_pixels, float pass);

// ---------------------------------------------------------------- progressive passes + output ----
// The CLI's pass loop (src/bin/raysnail.rs:311-427, parse_and_render): `passes` frames of
// `samples` spp at `depth`, each combined into the running image with combine_pixels; after each
// pass the noise map (calc_noise >= 0.01 on the combined image) is computed on the GPU and
// reported. Upstream the redo map never reaches the PixelController (the RedoController is built
// from the initial all-ones map before the loop, raysnail.rs:369-372), so every pass renders
// every pixel; `adaptive = true` applies each pass's map to the next pass instead.
struct PassReport {
    float noise_min = 0.f, noise_max = 0.f;  // raysnail.rs:394-407
    uint64_t oversample = 0;                  // pixels the redo map marks (raysnail.rs:411-422)
    rs_render_stats stats{};
};
struct ProgressiveResult {
    std::vector<Pixel> pixels;
    std::vector<PassReport> passes;
};
ProgressiveResult render_passes(const Camera& camera, World& world, size_t samples, size_t passes, uint64_t seed,
                                bool adaptive = false, size_t depth = 8);

// raysnail.rs:429-441: clamp(c, 0..1) * 255.5 -> u8, RGB rows top first
std::vector<uint8_t> quantize_rgb8(const std::vector<Pixel>& pixels);
// 8-bit RGB PNG (stored deflate blocks: no compression library needed); throws Error on I/O failure
void write_png(const std::string& path, size_t width, size_t height, const std::vector<uint8_t>& rgb);

// -------------------------------------------------------------------------------------- SDL ----
struct CameraData {  // src/sdl_parser.rs:52-57
    Vec3 location, look_at;
    double fov_angle = 60.0;
};
struct LightData {  // src/sdl_parser.rs:59-63
    Vec3 location;
    Color color;
};
struct SceneData {  // src/sdl_parser.rs:34-50
    std::optional<CameraData> camera;
    HittableList hittables;
    std::vector<LightData> lights;
};

struct SdlParser {  // src/sdl_parser.rs:180-205
    static SceneData parse(const std::string& filename);            // throws Error("Parse error") like Err(..)
    static SceneData parse_text(const std::string& text);
};

// The CLI's SDL conventions (src/bin/raysnail.rs:340-373): camera aperture 0.01, focus 10; each
// light -> Sphere(location, 12, DiffuseLight(color) x1.7) added to world and lights; gradient sky.
struct CliScene {
    Camera camera;
    World world;
};
CliScene cli_scene(SceneData scene, size_t width, size_t height);

}  // namespace raysnail

// C entry points of libraysnail_host for foreign callers and tests: build an SDL file's CLI scene
// into any sink table (e.g. the CPU oracle) or render it on the GPU through the C++ API.
extern "C" {
int rsh_sdl_build(const char* path, uint32_t width, uint32_t height, const raysnail::rsh_sink_api* api, void* scene,
                  rs_camera_desc* cam_out);
int rsh_sdl_render(const char* path, uint32_t width, uint32_t height, const rs_render_settings* st, float* out_rgba,
                   rs_render_stats* stats);
/* The CLI's pass loop on an SDL scene (render_passes): the combined RGBA image, and per pass
 * [noise_min, noise_max, oversample count] in noise_out (3 * passes floats; may be NULL). */
int rsh_sdl_render_passes(const char* path, uint32_t width, uint32_t height, uint32_t samples, uint32_t passes,
                          uint64_t seed, int adaptive, float* out_rgba, float* noise_out);
/* TriangleMesh::load: *n triangles, *pos and *nrm = malloc'd 9 doubles per triangle (free with rsh_free) */
int rsh_obj_load(const char* path, double scale, const double offset[3], double rotation_angle, int axis,
                 uint32_t* n, double** pos, double** nrm);
/* Perlin::new(point_count, vector, FastRng(seed)): values (3 or 1 per point) and perm_x|perm_y|perm_z */
int rsh_perlin_tables(uint64_t seed, uint32_t point_count, int vector, double* values, uint32_t* perms);
/* Image::new: decoded 8-bit RGB (*rgb malloc'd, free with rsh_free) */
int rsh_png_load(const char* path, uint32_t* width, uint32_t* height, uint8_t** rgb);
void rsh_free(void* p);
/* quantize_rgb8 + write_png of a W*H RGBA f32 image */
int rsh_write_png(const char* path, const float* rgba, uint32_t width, uint32_t height);
const char* rsh_last_error(void);
}
