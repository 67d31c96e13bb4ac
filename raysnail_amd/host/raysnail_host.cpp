// libraysnail_host: the C++ host layer (include/raysnail.hpp) over the C-ABI of libraysnail_hip.
// Object export, World / Camera / TakePhotoSettings, combine_pixels, and the C entry points.
// The SDL front end lives in sdl_parser.cpp.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
#include <string>

#include "raysnail.hpp"

namespace raysnail {

namespace {
thread_local std::string g_error;

rs_texture_desc tex_desc(SceneSink& sink, const Texture& t) {
    rs_texture_desc d;
    std::memset(&d, 0, sizeof(d));
    d.kind = t.kind;
    d.data = sink.texture_data(t);
    const float e[4] = {t.even.r, t.even.g, t.even.b, t.even.a};
    const float o[4] = {t.odd.r, t.odd.g, t.odd.b, t.odd.a};
    std::memcpy(d.even, e, sizeof(e));
    std::memcpy(d.odd, o, sizeof(o));
    d.scale = t.kind == RS_TEX_SOLID ? 1.0 : t.scale;
    return d;
}

// rs_* take rs_scene*; the sink table is typed on void* so oracle tables fit the same slots.
rs_scene* S(void* s) { return static_cast<rs_scene*>(s); }
const rsh_sink_api kHipApi = {
    [](void* s, const rs_material_desc* d, int32_t* id) { return rs_material(S(s), d, id); },
    [](void* s, const double* c, double r, const double* v, int32_t m, uint32_t* h) { return rs_sphere(S(s), c, r, v, m, h); },
    [](void* s, int32_t p, double k, double a0, double a1, double b0, double b1, int32_t m, uint32_t* h) {
        return rs_aarect(S(s), p, k, a0, a1, b0, b1, m, h);
    },
    [](void* s, const double* p0, const double* p1, int32_t m, uint32_t* h) { return rs_box(S(s), p0, p1, m, h); },
    [](void* s, const double* q, int32_t m, uint32_t* h) { return rs_quadric(S(s), q, m, h); },
    [](void* s, const double* p, const double* n, uint32_t c, int32_t m, uint32_t* f) { return rs_triangles(S(s), p, n, c, m, f); },
    [](void* s, uint32_t a, uint32_t b, int32_t m, uint32_t* h) { return rs_intersection(S(s), a, b, m, h); },
    [](void* s, uint32_t a, uint32_t b, int32_t m, uint32_t* h) { return rs_difference(S(s), a, b, m, h); },
    [](void* s, uint32_t o, const rs_transform* t, uint32_t n, uint32_t* h) { return rs_transformed(S(s), o, t, n, h); },
    [](void* s, uint32_t h) { return rs_world_add(S(s), h); },
    [](void* s, uint32_t h) { return rs_lights_add(S(s), h); },
    [](void* s, const float* lo, const float* hi) { return rs_set_background(S(s), lo, hi); },
    [](void* s, double t0, double t1) { return rs_set_time_range(S(s), t0, t1); },
    [](void* s, const rs_perlin_desc* d, int32_t* id) { return rs_perlin(S(s), d, id); },
    [](void* s, const uint8_t* rgb, uint32_t w, uint32_t h, int32_t* id) { return rs_image(S(s), rgb, w, h, id); },
    [](void* s, uint32_t b, const float* c, double d, uint32_t* h) { return rs_constant_medium(S(s), b, c, d, h); },
    []() { return rs_last_error(); },
};

void check_rs(int rc) {
    if (rc != RS_OK) throw Error(rc, rs_last_error());
}
}  // namespace

const rsh_sink_api& hip_sink_api() { return kHipApi; }

void SceneSink::check(int rc) const {
    if (rc != RS_OK) throw Error(rc, api.last_error ? api.last_error() : "scene sink error");
}

int32_t SceneSink::material(const MaterialRef& m) {
    if (!m) return RS_NO_MATERIAL;
    auto it = materials.find(m.get());
    if (it != materials.end()) return it->second;
    const int32_t id = m->export_to(*this);
    materials.emplace(m.get(), id);
    return id;
}

std::vector<uint32_t> SceneSink::object(const HittableRef& o) {
    if (!o) throw Error(RS_E_INVALID, "null hittable");
    auto it = objects.find(o.get());
    if (it != objects.end()) return it->second;
    std::vector<uint32_t> h = o->export_to(*this);
    objects.emplace(o.get(), h);
    return h;
}

int32_t SceneSink::texture_data(const Texture& t) {
    const void* key = t.kind == RS_TEX_PERLIN ? (const void*)t.perlin.get() : t.kind == RS_TEX_IMAGE ? (const void*)t.image.get() : nullptr;
    if (!key) {
        if (t.kind == RS_TEX_PERLIN || t.kind == RS_TEX_IMAGE) throw Error(RS_E_INVALID, "texture without data");
        return 0;
    }
    auto it = textures.find(key);
    if (it != textures.end()) return it->second;
    int32_t id = -1;
    if (t.kind == RS_TEX_PERLIN) {
        const PerlinData& p = *t.perlin;
        rs_perlin_desc d;
        std::memset(&d, 0, sizeof(d));
        d.point_count = p.point_count; d.vector = p.vector ? 1 : 0; d.smooth = (int32_t)p.smooth; d.type = p.type;
        d.depth = p.depth; d.scale = p.scale;
        d.values = p.values.data(); d.perm_x = p.perm_x.data(); d.perm_y = p.perm_y.data(); d.perm_z = p.perm_z.data();
        check(api.perlin(scene, &d, &id));
    } else {
        check(api.image(scene, t.image->rgb.data(), t.image->width, t.image->height, &id));
    }
    textures.emplace(key, id);
    return id;
}

// ---------------------------------------------------------------------------------- materials ----
rs_material_desc Material::base_desc(SceneSink& sink, int32_t kind, const Texture& t) const {
    rs_material_desc d;
    std::memset(&d, 0, sizeof(d));
    d.kind = kind;
    d.texture = tex_desc(sink, t);
    d.refractive = 1.0;
    d.exponent = 0.0;
    d.multiplier = 1.0;
    d.mix_p = 0.5;
    d.phong_factor = settings_.phong_factor;
    d.phong_exponent = settings_.phong_exponent;
    return d;
}

static int32_t add_material(SceneSink& sink, const rs_material_desc& d) {
    int32_t id = -1;
    sink.check(sink.api.material(sink.scene, &d, &id));
    return id;
}

int32_t Lambertian::export_to(SceneSink& sink) const { return add_material(sink, base_desc(sink, RS_MAT_LAMBERTIAN, tex_)); }
int32_t Metal::export_to(SceneSink& sink) const { return add_material(sink, base_desc(sink, RS_MAT_METAL, tex_)); }
int32_t Isotropic::export_to(SceneSink& sink) const {
    return add_material(sink, base_desc(sink, RS_MAT_ISOTROPIC, Texture::color(color_)));
}
int32_t BlinnPhong::export_to(SceneSink& sink) const {
    rs_material_desc d = base_desc(sink, RS_MAT_BLINN_PHONG, tex_);
    d.k_specular = k_;
    d.exponent = e_;
    return add_material(sink, d);
}
int32_t DiffuseMetal::export_to(SceneSink& sink) const {
    rs_material_desc d = base_desc(sink, RS_MAT_DIFFUSE_METAL, tex_);
    d.exponent = exponent_;
    return add_material(sink, d);
}
int32_t Dielectric::export_to(SceneSink& sink) const {
    rs_material_desc d = base_desc(sink, RS_MAT_DIELECTRIC, Texture::color(color_));
    d.refractive = refractive_;
    d.glass = glass_ ? 1 : 0;
    return add_material(sink, d);
}
int32_t DiffuseLight::export_to(SceneSink& sink) const {
    rs_material_desc d = base_desc(sink, RS_MAT_DIFFUSE_LIGHT, tex_);
    d.multiplier = mult_;
    return add_material(sink, d);
}
int32_t MixedMaterial::export_to(SceneSink& sink) const {
    const int32_t a = sink.material(m1_), b = sink.material(m2_);
    rs_material_desc d = base_desc(sink, RS_MAT_MIXED, Texture::color(Color{0.f, 0.f, 0.f, 1.f}));
    d.mix_a = a;
    d.mix_b = b;
    d.mix_p = p_;
    d.phong_factor = 0.0;   // unused: the library resolves the mix first and shades with the chosen
    d.phong_exponent = 0;   // material's own settings
    return add_material(sink, d);
}

// ----------------------------------------------------------------------------------- geometry ----
AARectMetrics::AARectMetrics(double k_, std::pair<double, double> a_, std::pair<double, double> b_)
    : k(k_), a(a_), b(b_) {
    if (!(a.first < a.second) || !(b.first < b.second))  // rect.rs:27-28 assert!
        throw Error(RS_E_INVALID, "AARectMetrics requires a0 < a1 and b0 < b1");
}

TriangleMesh::TriangleMesh(std::vector<double> positions, std::vector<double> normals, MaterialRef mat)
    : pos_(std::move(positions)), nrm_(std::move(normals)), mat_(std::move(mat)) {
    if (pos_.size() % 9 != 0 || (!nrm_.empty() && nrm_.size() != pos_.size()))
        throw Error(RS_E_INVALID, "TriangleMesh: 9 doubles per triangle for positions (and normals)");
}

std::vector<uint32_t> Sphere::export_to(SceneSink& sink) const {
    const double c[3] = {c_.x, c_.y, c_.z}, v[3] = {speed_.x, speed_.y, speed_.z};
    uint32_t h = 0;
    sink.check(sink.api.sphere(sink.scene, c, r_, v, sink.material(mat_), &h));
    return {h};
}

std::vector<uint32_t> AARect::export_to(SceneSink& sink) const {
    uint32_t h = 0;
    sink.check(sink.api.aarect(sink.scene, plane_, m_.k, m_.a.first, m_.a.second, m_.b.first, m_.b.second,
                               sink.material(mat_), &h));
    return {h};
}

std::vector<uint32_t> Box::export_to(SceneSink& sink) const {
    const double a[3] = {p0_.x, p0_.y, p0_.z}, b[3] = {p1_.x, p1_.y, p1_.z};
    uint32_t h = 0;
    sink.check(sink.api.box(sink.scene, a, b, sink.material(mat_), &h));
    return {h};
}

std::vector<uint32_t> Quadric::export_to(SceneSink& sink) const {
    uint32_t h = 0;
    sink.check(sink.api.quadric(sink.scene, q_.data(), sink.material(mat_), &h));
    return {h};
}

std::vector<uint32_t> TriangleMesh::export_to(SceneSink& sink) const {
    const uint32_t n = (uint32_t)(pos_.size() / 9);
    uint32_t first = 0;
    sink.check(sink.api.triangles(sink.scene, pos_.data(), nrm_.empty() ? nullptr : nrm_.data(), n,
                                  sink.material(mat_), &first));
    std::vector<uint32_t> h(n);
    for (uint32_t i = 0; i < n; ++i) h[i] = first + i;
    return h;
}

static uint32_t single(const std::vector<uint32_t>& h, const char* what) {
    if (h.size() != 1) throw Error(RS_E_UNSUPPORTED, std::string(what) + ": operand must be a single object");
    return h[0];
}

std::vector<uint32_t> Intersection::export_to(SceneSink& sink) const {
    const uint32_t a = single(sink.object(o1_), "Intersection"), b = single(sink.object(o2_), "Intersection");
    uint32_t h = 0;
    sink.check(sink.api.intersection(sink.scene, a, b, sink.material(mat_), &h));
    return {h};
}

std::vector<uint32_t> Difference::export_to(SceneSink& sink) const {
    const uint32_t a = single(sink.object(plus_), "Difference"), b = single(sink.object(minus_), "Difference");
    uint32_t h = 0;
    sink.check(sink.api.difference(sink.scene, a, b, sink.material(mat_), &h));
    return {h};
}

std::vector<uint32_t> ConstantMedium::export_to(SceneSink& sink) const {
    const uint32_t b = single(sink.object(boundary_), "ConstantMedium");
    const float c[4] = {color_.r, color_.g, color_.b, color_.a};
    uint32_t h = 0;
    sink.check(sink.api.constant_medium(sink.scene, b, c, density_, &h));
    return {h};
}

BVH::BVH(const HittableList& list, std::pair<double, double>) : objects_(list.objects()) {}

std::vector<uint32_t> BVH::export_to(SceneSink& sink) const {
    std::vector<uint32_t> out;
    for (const HittableRef& o : objects_)
        for (uint32_t h : sink.object(o)) out.push_back(h);
    return out;
}

std::vector<uint32_t> TfFacade::export_to(SceneSink& sink) const {
    const std::vector<uint32_t> child = sink.object(obj_);
    std::vector<uint32_t> out;
    for (uint32_t c : child) {  // a transformed mesh is a transformed triangle each
        uint32_t h = 0;
        sink.check(sink.api.transformed(sink.scene, c, stack_.items().data(), (uint32_t)stack_.len(), &h));
        out.push_back(h);
    }
    return out;
}

// -------------------------------------------------------------------------------------- World ----
World::World(HittableList hittables, HittableList lights, Gradient background, std::pair<double, double> time_range)
    : hittables_(std::move(hittables)), lights_(std::move(lights)), background_(background), time_range_(time_range) {}

World::~World() {
    if (scene_) rs_scene_destroy(scene_);
}

World::World(World&& o) noexcept
    : hittables_(std::move(o.hittables_)), lights_(std::move(o.lights_)), background_(o.background_),
      time_range_(o.time_range_), scene_(o.scene_) {
    o.scene_ = nullptr;
}

World& World::operator=(World&& o) noexcept {
    if (this != &o) {
        if (scene_) rs_scene_destroy(scene_);
        hittables_ = std::move(o.hittables_);
        lights_ = std::move(o.lights_);
        background_ = o.background_;
        time_range_ = o.time_range_;
        scene_ = o.scene_;
        o.scene_ = nullptr;
    }
    return *this;
}

void World::export_to(SceneSink& sink) const {
    const float lo[3] = {background_.lo.r, background_.lo.g, background_.lo.b};
    const float hi[3] = {background_.hi.r, background_.hi.g, background_.hi.b};
    sink.check(sink.api.set_background(sink.scene, lo, hi));
    sink.check(sink.api.set_time_range(sink.scene, time_range_.first, time_range_.second));
    for (const HittableRef& o : hittables_.objects())
        for (uint32_t h : sink.object(o)) sink.check(sink.api.world_add(sink.scene, h));
    for (const HittableRef& o : lights_.objects())
        for (uint32_t h : sink.object(o)) sink.check(sink.api.lights_add(sink.scene, h));
}

rs_scene* World::device_scene() {
    if (scene_) return scene_;
    rs_scene* s = nullptr;
    check_rs(rs_scene_create(&s));
    try {
        SceneSink sink(hip_sink_api(), s);
        export_to(sink);
        check_rs(rs_scene_commit(s));
    } catch (...) {
        rs_scene_destroy(s);
        throw;
    }
    scene_ = s;
    return scene_;
}

// ------------------------------------------------------------------------------------- Camera ----
CameraBuilder::CameraBuilder() {
    std::memset(&d_, 0, sizeof(d_));
    d_.look_at[2] = -1.0;
    d_.vup[1] = 1.0;
    d_.fov = 90.0;
    d_.aperture = 0.0;
    d_.focus = 1.0;
    d_.shutter = 0.0;
    d_.width = 400;
    d_.height = 200;
}

CameraBuilder& CameraBuilder::focus_to_look_at() {  // camera.rs: (look_at - look_from).length()
    const double dx = d_.look_at[0] - d_.look_from[0], dy = d_.look_at[1] - d_.look_from[1],
                 dz = d_.look_at[2] - d_.look_from[2];
    d_.focus = std::sqrt(std::fma(dz, dz, std::fma(dx, dx, dy * dy)));  // length_squared, vec3.rs:152-160
    return *this;
}

rs_render_settings TakePhotoSettings::settings() const {
    rs_render_settings st;
    std::memset(&st, 0, sizeof(st));
    st.samples = samples_;
    st.depth = depth_;
    st.gamma = gamma_ ? 1 : 0;
    st.mode = mode_;
    st.seed = seed_;
    st.pass = pass_;
    st.row_begin = row_begin_;
    st.row_end = row_end_;
    st.row_step = row_step_;
    return st;
}

std::vector<Pixel> TakePhotoSettings::shot_to_target(const char*, World& world, PainterTarget* target,
                                                     PainterController*, const PixelController* pixel_map) {
    const rs_camera_desc& cam = camera_.desc();
    const size_t W = cam.width, H = cam.height;
    std::vector<uint8_t> mask;
    if (pixel_map) {
        mask.resize(W * H);
        for (size_t y = 0; y < H; ++y)
            for (size_t x = 0; x < W; ++x) mask[y * W + x] = pixel_map->calculate_pixel(x, y) ? 1 : 0;
    }
    std::vector<Pixel> out(W * H, Pixel{0.f, 0.f, 0.f, 0.f});
    const rs_render_settings st = settings();
    const uint8_t* mp = mask.empty() ? nullptr : mask.data();
    if (!target) {
        check_rs(rs_render(world.device_scene(), &cam, &st, mp, reinterpret_cast<float*>(out.data()), &stats_));
        return out;
    }
    // Progressive delivery: upstream's workers call register_pixels as each row finishes
    // (painter.rs:214), which feeds the CLI preview. rs_render_rows renders the frame's row lattice in
    // bands, several in flight, and hands each band's rows over as soon as the band is complete, while
    // the later bands are traced; pixels do not depend on the banding (every sample has its own RNG
    // stream), so the frame is the one-call frame. Rows off the lattice (untouched, all zero) are
    // registered before the end-of-pass sentinel (painter.rs:332).
    struct Ctx {
        PainterTarget* target;
        size_t W, H;
        std::vector<uint8_t> sent;
        const std::vector<Pixel>* out;
        std::exception_ptr err;
    } ctx{target, W, H, std::vector<uint8_t>(H, 0), &out, nullptr};
    rs_row_callback cb = [](void* u, uint32_t y, const float* row, uint32_t w) {
        Ctx& c = *static_cast<Ctx*>(u);
        if (c.err) return;
        try {  // (no exception may cross the C ABI: kept and rethrown after the call)
            if (y == c.H) {
                for (size_t r = 0; r < c.H; ++r)
                    if (!c.sent[r]) c.target->register_pixels(r, std::vector<Pixel>(c.out->begin() + r * c.W, c.out->begin() + (r + 1) * c.W));
                c.target->register_pixels(c.H, {});
                return;
            }
            c.sent[y] = 1;
            std::vector<Pixel> px(w);
            std::memcpy(px.data(), row, (size_t)w * sizeof(Pixel));
            c.target->register_pixels(y, px);
        } catch (...) {
            c.err = std::current_exception();
        }
    };
    stats_ = rs_render_stats{};
    check_rs(rs_render_rows(world.device_scene(), &cam, &st, mp, reinterpret_cast<float*>(out.data()), 16, cb, &ctx, &stats_));
    if (ctx.err) std::rethrow_exception(ctx.err);
    return out;
}

void combine_pixels(std::vector<Pixel>& old_pixels, const std::vector<Pixel>& new_pixels, float p) {
    if (old_pixels.size() != new_pixels.size()) throw Error(RS_E_INVALID, "combine_pixels: size mismatch");
    for (size_t i = 0; i < new_pixels.size(); ++i) {
        const Pixel& n = new_pixels[i];
        if (n[0] == 0.f && n[1] == 0.f && n[2] == 0.f && n[3] == 0.f) continue;  // keep old
        Pixel& o = old_pixels[i];
        const float d = p + 1.0f;
        for (int c = 0; c < 4; ++c) o[c] = (o[c] * p + n[c]) / d;
    }
}

ProgressiveResult render_passes(const Camera& camera, World& world, size_t samples, size_t passes, uint64_t seed,
                                bool adaptive, size_t depth) {
    const size_t W = camera.picture_width(), H = camera.picture_height();
    ProgressiveResult res;
    res.pixels.assign(W * H, Pixel{0.f, 0.f, 0.f, 1.f});  // raysnail.rs:317-322
    std::vector<uint8_t> redo(W * H, 1);
    struct Redo : PixelController {  // RedoController, raysnail.rs:123-134
        const std::vector<uint8_t>* map;
        size_t width;
        bool calculate_pixel(size_t x, size_t y) const override { return (*map)[y * width + x] > 0; }
    } controller;
    controller.map = &redo;
    controller.width = W;
    const std::vector<uint8_t> initial = redo;  // what upstream's controller keeps seeing
    for (size_t p = 0; p < passes; ++p) {
        TakePhotoSettings photo = camera.take_photo();
        photo.samples(samples).depth(depth).seed(seed).pass_index((uint32_t)p);
        if (!adaptive) controller.map = &initial;
        std::vector<Pixel> px = photo.shot_to_target(nullptr, world, nullptr, nullptr, &controller);
        combine_pixels(res.pixels, px, (float)p);
        PassReport rep;
        rep.stats = photo.last_stats();
        rs_noise_stats ns{};
        check_rs(rs_noise_map(reinterpret_cast<const float*>(res.pixels.data()), (uint32_t)W, (uint32_t)H, 0.01f,
                              redo.data(), &ns));
        rep.noise_min = ns.min;
        rep.noise_max = ns.max;
        rep.oversample = ns.count;
        res.passes.push_back(rep);
        controller.map = &redo;
    }
    return res;
}

std::vector<uint8_t> quantize_rgb8(const std::vector<Pixel>& pixels) {
    std::vector<uint8_t> out(pixels.size() * 3);
    for (size_t i = 0; i < pixels.size(); ++i)
        for (int c = 0; c < 3; ++c) {
            double v = (double)pixels[i][c];  // clamp(c as f64, 0.0 .. 1.0) * 255.5, `as u8` saturates
            v = v < 0.0 ? 0.0 : v > 1.0 ? 1.0 : v;
            if (v != v) v = 0.0;              // Rust's float -> int cast maps NaN to 0
            const double q = v * 255.5;
            out[3 * i + c] = (uint8_t)(q >= 255.0 ? 255 : (int)q);
        }
    return out;
}

namespace {
uint32_t crc32_of(const uint8_t* p, size_t n, uint32_t c = 0xFFFFFFFFu) {
    static uint32_t table[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t k = i;
            for (int j = 0; j < 8; ++j) k = (k & 1) ? 0xEDB88320u ^ (k >> 1) : k >> 1;
            table[i] = k;
        }
        init = true;
    }
    for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return c;
}
void put_be32(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back((uint8_t)(x >> 24)); v.push_back((uint8_t)(x >> 16)); v.push_back((uint8_t)(x >> 8)); v.push_back((uint8_t)x);
}
void chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
    put_be32(out, (uint32_t)data.size());
    std::vector<uint8_t> td(type, type + 4);
    td.insert(td.end(), data.begin(), data.end());
    out.insert(out.end(), td.begin(), td.end());
    put_be32(out, crc32_of(td.data(), td.size()) ^ 0xFFFFFFFFu);
}
}  // namespace

void write_png(const std::string& path, size_t width, size_t height, const std::vector<uint8_t>& rgb) {
    if (rgb.size() != width * height * 3) throw Error(RS_E_INVALID, "write_png: size mismatch");
    std::vector<uint8_t> raw;  // filter byte 0 + row
    raw.reserve(height * (width * 3 + 1));
    for (size_t y = 0; y < height; ++y) {
        raw.push_back(0);
        raw.insert(raw.end(), rgb.begin() + y * width * 3, rgb.begin() + (y + 1) * width * 3);
    }
    std::vector<uint8_t> z = {0x78, 0x01};  // zlib header, stored blocks of <= 65535 bytes
    uint32_t a = 1, b = 0;
    for (size_t i = 0; i < raw.size(); i += 65535) {
        const size_t n = std::min<size_t>(65535, raw.size() - i);
        z.push_back(i + n >= raw.size() ? 1 : 0);
        z.push_back((uint8_t)n); z.push_back((uint8_t)(n >> 8));
        z.push_back((uint8_t)~n); z.push_back((uint8_t)(~n >> 8));
        z.insert(z.end(), raw.begin() + i, raw.begin() + i + n);
    }
    for (uint8_t c : raw) { a = (a + c) % 65521; b = (b + a) % 65521; }  // adler32
    put_be32(z, (b << 16) | a);
    std::vector<uint8_t> png = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1A, '\n'};
    std::vector<uint8_t> ihdr;
    put_be32(ihdr, (uint32_t)width);
    put_be32(ihdr, (uint32_t)height);
    ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});  // 8-bit RGB
    chunk(png, "IHDR", ihdr);
    chunk(png, "IDAT", z);
    chunk(png, "IEND", {});
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) throw Error(RS_E_INVALID, "cannot write " + path);
    const size_t wr = std::fwrite(png.data(), 1, png.size(), f);
    std::fclose(f);
    if (wr != png.size()) throw Error(RS_E_INVALID, "short write to " + path);
}

CliScene cli_scene(SceneData scene, size_t width, size_t height) {
    if (!scene.camera) throw Error(RS_E_INVALID, "scene has no camera");  // scene_data.camera.unwrap()
    const CameraData& cd = *scene.camera;
    Camera camera = CameraBuilder()
                        .look_from(cd.location)
                        .look_at(cd.look_at)
                        .fov(cd.fov_angle)
                        .aperture(0.01)
                        .focus(10.0)
                        .width(width)
                        .height(height)
                        .build();
    HittableList lights;
    for (const LightData& l : scene.lights) {
        auto mat = std::make_shared<DiffuseLight>(Texture::color(l.color));
        mat->multiplier(1.7);
        auto s1 = std::make_shared<Sphere>(l.location, 12.0, mat);
        auto s2 = std::make_shared<Sphere>(*s1);  // rs.clone() into lights, rs into the world list
        lights.add(s1);
        scene.hittables.add(s2);
    }
    Gradient bg{Color{0.3f, 0.4f, 0.5f, 1.f}, Color{0.7f, 0.89f, 1.0f, 1.f}};
    World world(std::move(scene.hittables), std::move(lights), bg, {0.0, camera.shutter_speed()});
    return CliScene{camera, std::move(world)};
}

namespace detail {
void set_error(const std::string& e) { g_error = e; }
const char* last_error() { return g_error.c_str(); }
}

}  // namespace raysnail

using namespace raysnail;

template <class F>
static int guarded(F&& f) {
    try {
        f();
        detail::set_error("");
        return RS_OK;
    } catch (const Error& e) {
        detail::set_error(e.what());
        return e.code() ? e.code() : RS_E_INVALID;
    } catch (const std::exception& e) {
        detail::set_error(e.what());
        return RS_E_INVALID;
    }
}

extern "C" int rsh_sdl_build(const char* path, uint32_t width, uint32_t height, const rsh_sink_api* api, void* scene,
                             rs_camera_desc* cam_out) {
    return guarded([&] {
        if (!path || !api || !scene) throw Error(RS_E_INVALID, "null argument");
        CliScene sc = cli_scene(SdlParser::parse(path), width, height);
        SceneSink sink(*api, scene);
        sc.world.export_to(sink);
        if (cam_out) *cam_out = sc.camera.desc();
    });
}

extern "C" int rsh_sdl_render(const char* path, uint32_t width, uint32_t height, const rs_render_settings* st,
                              float* out_rgba, rs_render_stats* stats) {
    return guarded([&] {
        if (!path || !st || !out_rgba) throw Error(RS_E_INVALID, "null argument");
        CliScene sc = cli_scene(SdlParser::parse(path), width, height);
        TakePhotoSettings photo = sc.camera.take_photo();
        photo.samples(st->samples).depth(st->depth).gamma(st->gamma != 0).seed(st->seed).pass_index(st->pass)
            .rows(st->row_begin, st->row_end, st->row_step).mode(st->mode);
        std::vector<Pixel> px = photo.shot(nullptr, sc.world);
        std::memcpy(out_rgba, px.data(), px.size() * sizeof(Pixel));
        if (stats) *stats = photo.last_stats();
    });
}

extern "C" int rsh_sdl_render_passes(const char* path, uint32_t width, uint32_t height, uint32_t samples,
                                     uint32_t passes, uint64_t seed, int adaptive, float* out_rgba, float* noise_out) {
    return guarded([&] {
        if (!path || !out_rgba) throw Error(RS_E_INVALID, "null argument");
        CliScene sc = cli_scene(SdlParser::parse(path), width, height);
        ProgressiveResult r = render_passes(sc.camera, sc.world, samples, passes, seed, adaptive != 0);
        std::memcpy(out_rgba, r.pixels.data(), r.pixels.size() * sizeof(Pixel));
        if (noise_out)
            for (size_t p = 0; p < r.passes.size(); ++p) {
                noise_out[3 * p] = r.passes[p].noise_min;
                noise_out[3 * p + 1] = r.passes[p].noise_max;
                noise_out[3 * p + 2] = (float)r.passes[p].oversample;
            }
    });
}

extern "C" int rsh_write_png(const char* path, const float* rgba, uint32_t width, uint32_t height) {
    return guarded([&] {
        if (!path || !rgba) throw Error(RS_E_INVALID, "null argument");
        std::vector<Pixel> px((size_t)width * height);
        std::memcpy(px.data(), rgba, px.size() * sizeof(Pixel));
        write_png(path, width, height, quantize_rgb8(px));
    });
}

extern "C" const char* rsh_last_error(void) { return detail::last_error(); }
