// C++ host API end to end on the GPU (run by tests/test_gpu_host.py): a scene built from the
// raysnail-shaped classes (every material, sphere / moving sphere / rect / box / quadric / mesh /
// intersection / difference / transforms), rendered through TakePhotoSettings::shot_to_target with
// a PainterTarget and a PixelController, and checked bit for bit against the CPU oracle, which is
// filled through the same export routine (World::export_to) with the oracle's sink table.
// usage: test_api <path to oracle/build/liboracle.so>
#include <dlfcn.h>

#include <cmath>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "raysnail.hpp"

using namespace raysnail;

static int failures = 0;
#define CHECK(cond, ...)                                   \
    do {                                                   \
        if (!(cond)) {                                     \
            std::printf("FAIL %s:%d: ", __FILE__, __LINE__); \
            std::printf(__VA_ARGS__);                      \
            std::printf("\n");                             \
            ++failures;                                    \
        }                                                  \
    } while (0)

struct Oracle {
    void* so = nullptr;
    rsh_sink_api api{};
    void* (*create)() = nullptr;
    void (*destroy)(void*) = nullptr;
    int (*commit)(void*) = nullptr;
    int (*render)(void*, const rs_camera_desc*, const rs_render_settings*, const uint8_t*, float*, int,
                  rs_render_stats*) = nullptr;
    template <class T>
    void sym(T& f, const char* name) {
        f = reinterpret_cast<T>(dlsym(so, name));
        if (!f) { std::printf("missing oracle symbol %s\n", name); std::exit(2); }
    }
    explicit Oracle(const char* path) {
        so = dlopen(path, RTLD_NOW);
        if (!so) { std::printf("dlopen %s: %s\n", path, dlerror()); std::exit(2); }
        sym(api.material, "orc_material"); sym(api.sphere, "orc_sphere"); sym(api.aarect, "orc_aarect");
        sym(api.box, "orc_box"); sym(api.quadric, "orc_quadric"); sym(api.triangles, "orc_triangles");
        sym(api.intersection, "orc_intersection"); sym(api.difference, "orc_difference");
        sym(api.transformed, "orc_transformed"); sym(api.world_add, "orc_world_add");
        sym(api.lights_add, "orc_lights_add"); sym(api.set_background, "orc_set_background");
        sym(api.set_time_range, "orc_set_time_range"); sym(api.last_error, "orc_last_error");
        sym(create, "orc_scene_create"); sym(destroy, "orc_scene_destroy"); sym(commit, "orc_commit");
        sym(render, "orc_render");
    }
};

static Texture col(float r, float g, float b) { return Texture::color(Color{r, g, b, 1.f}); }

static World build_world() {
    HittableList objects, lights;
    auto ground = std::make_shared<Lambertian>(Texture::checker(Color{0.3f, 0.3f, 0.3f, 1.f}, Color{0.9f, 0.9f, 0.9f, 1.f}, 10.0));
    objects.add(std::make_shared<Sphere>(Point3{0, -1000, 0}, 1000, ground));
    auto glass = std::make_shared<Dielectric>(Color{1.f, 1.f, 1.f, 1.f}, 1.5);
    glass->reflect_curve(Glass{});
    objects.add(std::make_shared<Sphere>(Point3{0, 1, 0}, 1.0, glass));
    auto phong = std::make_shared<Lambertian>(col(0.4f, 0.2f, 0.1f));
    phong->set(CommonMaterialSettings{2.0, 8});
    auto moving = std::make_shared<Sphere>(Point3{-4, 1, 0}, 1.0, phong);
    moving->with_speed(Vec3{0, 0.3, 0});
    objects.add(moving);
    objects.add(std::make_shared<Sphere>(Point3{4, 1, 0}, 1.0, std::make_shared<Metal>(col(0.7f, 0.6f, 0.5f))));
    objects.add(std::make_shared<Sphere>(Point3{2, 0.4, 2}, 0.4, std::make_shared<DiffuseMetal>(250.0, col(0.8f, 0.8f, 0.2f))));
    auto mix = std::make_shared<MixedMaterial>(std::make_shared<Metal>(col(0.9f, 0.9f, 0.9f)),
                                               std::make_shared<Lambertian>(col(0.1f, 0.5f, 0.2f)), 0.3);
    objects.add(std::make_shared<Box>(Point3{-2.5, 0, 1.5}, Point3{-1.5, 0.8, 2.5}, mix));
    // CSG + transforms
    auto q = std::make_shared<Quadric>(1, 0, 0, 0, -1, 0, 0, 1, 0, -0.1, nullptr);
    auto clip = std::make_shared<Box>(Point3{-0.7, -0.7, -0.7}, Point3{0.7, 0.7, 0.7}, nullptr);
    TransformStack st;
    st.push(Transform::rotate_by_y_axis(0.4));
    st.push(Transform::translate(Vec3{1.5, 0.7, -2.0}));
    objects.add(std::make_shared<TfFacade>(std::make_shared<Intersection>(q, clip, std::make_shared<Lambertian>(col(0.8f, 0.3f, 0.5f))), st));
    auto cube = std::make_shared<Box>(Point3{-0.5, 0, -0.5}, Point3{0.5, 1, 0.5}, std::make_shared<Lambertian>(col(0.2f, 0.4f, 0.8f)));
    auto hole = std::make_shared<Sphere>(Point3{0, 1, 0}, 0.45, std::make_shared<Lambertian>(col(0.9f, 0.9f, 0.9f)));
    TransformStack st2;
    st2.push(Transform::scale(Vec3{1.2, 1.0, 1.2}));
    st2.push(Transform::translate(Vec3{-1.0, 0.0, -2.5}));
    objects.add(std::make_shared<TfFacade>(std::make_shared<Difference>(cube, hole, nullptr), st2));
    // a small mesh (tetrahedron), face normals
    std::vector<double> tri = {3, 0, -1, 3.5, 1, -1, 4, 0, -1,   3, 0, -1, 3.5, 0, -2, 3.5, 1, -1,
                               4, 0, -1, 3.5, 1, -1, 3.5, 0, -2,  3, 0, -1, 4, 0, -1, 3.5, 0, -2};
    objects.add(std::make_shared<TriangleMesh>(tri, std::vector<double>{}, std::make_shared<Lambertian>(col(0.6f, 0.6f, 0.1f))));
    // lights: a sphere and an xz rect, both in the world list too
    auto lamp = std::make_shared<DiffuseLight>(col(1.f, 0.9f, 0.7f));
    lamp->multiplier(4.0);
    auto sun = std::make_shared<Sphere>(Point3{30, 60, 20}, 12.0, lamp);
    auto panel = AARect::new_xz(AARectMetrics(8.0, {-1.0, 1.0}, {-1.0, 1.0}),
                                std::make_shared<DiffuseLight>(col(3.f, 3.f, 3.f)));
    objects.add(sun);
    objects.add(panel);
    lights.add(sun);
    lights.add(panel);
    return World(std::move(objects), std::move(lights), Gradient{}, {0.0, 1.0});
}

struct Rows : PainterTarget {
    std::vector<size_t> ys;
    size_t sentinel_len = 99;
    void register_pixels(size_t y, const std::vector<Pixel>& px) override {
        ys.push_back(y);
        sentinel_len = px.size();
    }
};

struct Checkerboard : PixelController {
    bool calculate_pixel(size_t x, size_t y) const override { return (x / 3 + y / 2) % 2 == 0; }
};

int main(int argc, char** argv) {
    if (argc < 2) { std::printf("usage: test_api liboracle.so\n"); return 2; }
    Oracle orc(argv[1]);
    const size_t W = 96, H = 60;
    Camera cam = CameraBuilder().look_from({8, 3, 6}).look_at({0, 0.6, 0}).fov(35).aperture(0.05)
                     .focus_to_look_at().shutter_speed(1.0).width(W).height(H).build();
    World world = build_world();

    // oracle, through the same export routine
    void* os = orc.create();
    SceneSink sink(orc.api, os);
    world.export_to(sink);
    CHECK(orc.commit(os) == 0, "oracle commit: %s", orc.api.last_error());

    for (int mode : {RS_MODE_AUTO, RS_MODE_MEGAKERNEL, RS_MODE_WAVEFRONT}) {
        TakePhotoSettings photo = cam.take_photo();
        photo.samples(16).depth(12).seed(77).mode(mode);
        Rows rows;
        Checkerboard mask;
        std::vector<Pixel> g = photo.shot_to_target(nullptr, world, &rows, nullptr, &mask);
        // PainterTarget: rows 0..H-1, then the (H, []) sentinel (painter.rs:332)
        CHECK(rows.ys.size() == H + 1 && rows.ys.back() == H && rows.sentinel_len == 0, "row callbacks");
        std::vector<uint8_t> m(W * H);
        for (size_t y = 0; y < H; ++y)
            for (size_t x = 0; x < W; ++x) m[y * W + x] = mask.calculate_pixel(x, y);
        std::vector<Pixel> o(W * H, Pixel{0, 0, 0, 0});
        rs_render_settings st = photo.settings();
        rs_render_stats ost{};
        CHECK(orc.render(os, &cam.desc(), &st, m.data(), reinterpret_cast<float*>(o.data()), 8, &ost) == 0, "oracle render");
        size_t same = 0, masked_zero = 0, n_masked = 0;
        for (size_t i = 0; i < W * H; ++i) {
            same += std::memcmp(&g[i], &o[i], sizeof(Pixel)) == 0;
            if (!m[i]) { ++n_masked; masked_zero += g[i][0] == 0 && g[i][1] == 0 && g[i][2] == 0 && g[i][3] == 0; }
        }
        CHECK(same == W * H, "mode %d: %zu/%zu pixels bitwise equal to the oracle", mode, same, W * H);
        CHECK(masked_zero == n_masked && n_masked > 0, "masked pixels are [0,0,0,0]");
        CHECK(photo.last_stats().segments == ost.segments, "segments %llu vs %llu",
              (unsigned long long)photo.last_stats().segments, (unsigned long long)ost.segments);
        std::printf("mode %d: %zu/%zu pixels equal, segments %llu\n", mode, same, W * H,
                    (unsigned long long)ost.segments);
    }

    // progressive delivery (painter.rs:214): rows arrive, in lattice order, while later bands of the
    // frame are still being traced; then the sentinel; the frame equals the one-call frame
    {
        Camera big = CameraBuilder().look_from({8, 3, 6}).look_at({0, 0.6, 0}).fov(35).aperture(0.05)
                         .focus_to_look_at().shutter_speed(1.0).width(480).height(270).build();
        TakePhotoSettings photo = big.take_photo();
        photo.samples(64).depth(12).seed(3);
        struct Timed : PainterTarget {
            std::chrono::steady_clock::time_point t0;
            std::vector<size_t> ys;
            std::vector<double> ms;
            void register_pixels(size_t y, const std::vector<Pixel>&) override {
                ys.push_back(y);
                ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
            }
        } tr;
        tr.t0 = std::chrono::steady_clock::now();
        std::vector<Pixel> g = photo.shot_to_target(nullptr, world, &tr, nullptr, nullptr);
        CHECK(tr.ys.size() == 271 && tr.ys.back() == 270, "progressive rows + sentinel");
        bool ordered = true;
        for (size_t y = 0; y < 270; ++y) ordered = ordered && tr.ys[y] == y;
        CHECK(ordered, "rows delivered in lattice order");
        CHECK(tr.ms[0] < 0.6 * tr.ms.back(), "first row at %.1f ms of a %.1f ms frame", tr.ms[0], tr.ms.back());
        std::vector<Pixel> one = photo.shot(nullptr, world);
        CHECK(std::memcmp(g.data(), one.data(), g.size() * sizeof(Pixel)) == 0, "banded frame == one-call frame");
        std::printf("progressive: first row at %.1f ms, sentinel at %.1f ms\n", tr.ms[0], tr.ms.back());
    }

    // progressive passes folded like the CLI (raysnail.rs:379-427)
    std::vector<Pixel> acc(W * H, Pixel{0, 0, 0, 1});
    std::vector<Pixel> acc_o = acc;
    for (uint32_t p = 0; p < 3; ++p) {
        TakePhotoSettings photo = cam.take_photo();
        photo.samples(4).depth(8).seed(5).pass_index(p);
        std::vector<Pixel> g = photo.shot(nullptr, world);
        combine_pixels(acc, g, (float)p);
        std::vector<Pixel> o(W * H, Pixel{0, 0, 0, 0});
        rs_render_settings st = photo.settings();
        rs_render_stats ost{};
        CHECK(orc.render(os, &cam.desc(), &st, nullptr, reinterpret_cast<float*>(o.data()), 8, &ost) == 0,
              "oracle render (pass %u)", p);
        size_t nd = 0, first = 0;
        for (size_t i = 0; i < W * H; ++i)
            if (std::memcmp(&g[i], &o[i], sizeof(Pixel)) != 0) { if (!nd) first = i; ++nd; }
        CHECK(nd == 0, "pass %u: %zu pixels differ, first (%zu,%zu) gpu %.9g %.9g %.9g oracle %.9g %.9g %.9g", p, nd,
              first % W, first / W, g[first][0], g[first][1], g[first][2], o[first][0], o[first][1], o[first][2]);
        combine_pixels(acc_o, o, (float)p);
    }
    CHECK(std::memcmp(acc.data(), acc_o.data(), acc.size() * sizeof(Pixel)) == 0, "combined passes differ");

    // errors surface as exceptions with the library's message
    bool threw = false;
    try {
        AARectMetrics bad(1.0, {1.0, 0.0}, {0.0, 1.0});
    } catch (const Error& e) {
        threw = e.code() == RS_E_INVALID;
    }
    CHECK(threw, "AARectMetrics a0 >= a1 must throw");
    HittableList no_lights;
    no_lights.add(std::make_shared<Sphere>(Point3{0, 0, 0}, 1.0, std::make_shared<Lambertian>(col(1, 1, 1))));
    World dark(std::move(no_lights), HittableList{});
    threw = false;
    try {
        dark.device_scene();
    } catch (const Error& e) {
        threw = e.code() == RS_E_NO_LIGHTS;
    }
    CHECK(threw, "a pdf material without lights must fail with RS_E_NO_LIGHTS");

    orc.destroy(os);
    std::printf(failures ? "FAILED (%d)\n" : "ALL OK\n", failures);
    return failures ? 1 : 0;
}
