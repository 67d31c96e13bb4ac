// scene_gen.cpp — TEST INFRASTRUCTURE ONLY (part of liboracle.so; see oracle.cpp's header).
//
// An independent C++ build of the RTIOW final scene (examples/rtow_13_1.rs:15-46 ->
// examples/common/ray_tracing_in_one_weekend.rs:8-20 -> examples/common/scene.rs:23-75, 133-191),
// written from the reference and the published algorithms of the crates it calls, so the oracle's
// RTIOW scene does not come from raysnail_amd/scenes.py (the Python generator the GPU tests feed):
//
//   SeedRandom::new(seed) = StdRng::seed_from_u64 (src/prelude/random.rs:82)
//     rand_core 0.6.2 seed_from_u64: PCG32 (MUL 6364136223846793005, INC 11634580027462260723),
//       one 32-bit output word per 4 key bytes, little-endian
//     rand 0.8.3 StdRng = rand_chacha 0.3.0 ChaCha12Rng: ChaCha with 12 rounds, 64-bit block counter
//       (words 12-13) from 0, stream 0 (words 14-15), rand_core BlockRng over 4-block (64-word) buffers
//   SeedRandom::normal = gen_range(0.0..=1.0) (random.rs:18-20): UniformFloat<f64>::new_inclusive
//     (scale shrunk until scale * max_rand + low <= high) then sample: value1_2 from the top 52 bits
//     of next_u64 with exponent 0, minus 1, times scale plus low
//   SeedRandom::range(a..b) (random.rs:23-25): UniformFloat::sample_single (first draw < b returned)
//
// No reference test pins these crates: the ChaCha core is checked against RFC 7539
// (20 rounds), the scene against the Python restatement and the committed digest (tests/).
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../include/raysnail_hip.h"

struct orc_scene;

extern "C" {
int orc_material(orc_scene* s, const rs_material_desc* d, int32_t* id_out);
int orc_sphere(orc_scene* s, const double c[3], double r, const double speed[3], int32_t mat, uint32_t* out);
int orc_world_add(orc_scene* s, uint32_t h);
int orc_lights_add(orc_scene* s, uint32_t h);
int orc_set_background(orc_scene* s, const float lo[3], const float hi[3]);
int orc_set_time_range(orc_scene* s, double t0, double t1);
}

namespace {

inline uint32_t rotl(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }

// ChaCha block function: 16 state words in, `rounds` rounds (pairs of column + diagonal), feed-forward
void chacha_block(const uint32_t in[16], int rounds, uint32_t out[16]) {
    uint32_t x[16];
    std::memcpy(x, in, sizeof(x));
    auto qr = [&x](int a, int b, int c, int d) {
        x[a] += x[b]; x[d] ^= x[a]; x[d] = rotl(x[d], 16);
        x[c] += x[d]; x[b] ^= x[c]; x[b] = rotl(x[b], 12);
        x[a] += x[b]; x[d] ^= x[a]; x[d] = rotl(x[d], 8);
        x[c] += x[d]; x[b] ^= x[c]; x[b] = rotl(x[b], 7);
    };
    for (int i = 0; i < rounds; i += 2) {
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15);
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14);
    }
    for (int i = 0; i < 16; ++i) out[i] = x[i] + in[i];
}

class StdRng {  // ChaCha12Rng behind BlockRng<ChaCha12Core>
public:
    explicit StdRng(uint64_t state) {
        const uint64_t MUL = 6364136223846793005ull, INC = 11634580027462260723ull;
        for (int i = 0; i < 8; ++i) {
            state = state * MUL + INC;
            const uint32_t xs = (uint32_t)(((state >> 18) ^ state) >> 27);
            const uint32_t rot = (uint32_t)(state >> 59);
            key_[i] = (xs >> rot) | (xs << ((32 - rot) & 31));
        }
    }
    uint64_t next_u64() {
        if (index_ < 63) {
            const uint64_t v = ((uint64_t)buf_[index_ + 1] << 32) | buf_[index_];
            index_ += 2;
            return v;
        }
        if (index_ >= 64) {
            refill();
            index_ = 2;
            return ((uint64_t)buf_[1] << 32) | buf_[0];
        }
        const uint64_t lo = buf_[63];
        refill();
        index_ = 1;
        return ((uint64_t)buf_[0] << 32) | lo;
    }

private:
    void refill() {
        for (int b = 0; b < 4; ++b) {
            uint32_t st[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
            for (int i = 0; i < 8; ++i) st[4 + i] = key_[i];
            const uint64_t ctr = counter_ + (uint64_t)b;
            st[12] = (uint32_t)ctr; st[13] = (uint32_t)(ctr >> 32);
            st[14] = 0; st[15] = 0;
            chacha_block(st, 12, buf_ + 16 * b);
        }
        counter_ += 4;
    }
    uint32_t key_[8];
    uint64_t counter_ = 0;
    uint32_t buf_[64];
    int index_ = 64;
};

double bits_to_double(uint64_t b) { double d; std::memcpy(&d, &b, 8); return d; }
double value0_1(StdRng& r) { return bits_to_double((1023ull << 52) | (r.next_u64() >> 12)) - 1.0; }
double next_down_positive(double x) { uint64_t b; std::memcpy(&b, &x, 8); return bits_to_double(b - 1); }

struct SeedRandom {
    StdRng rng;
    explicit SeedRandom(uint64_t seed) : rng(seed) {}
    double normal() {  // gen_range(0.0..=1.0)
        const double low = 0.0, high = 1.0;
        const double max_rand = bits_to_double((1023ull << 52) | (UINT64_MAX >> 12)) - 1.0;
        double scale = (high - low) / max_rand;
        while (scale * max_rand + low > high) scale = next_down_positive(scale);
        return value0_1(rng) * scale + low;
    }
    double range(double low, double high) {  // gen_range(low..high)
        double scale = high - low;
        for (;;) {
            const double res = value0_1(rng) * scale + low;
            if (res < high) return res;
            scale = next_down_positive(scale);
        }
    }
};

// one sphere of the generated list
struct Ball {
    double c[3], r;
    int kind;          // RS_MAT_* ; the ground is RS_MAT_LAMBERTIAN with checker = 1
    int checker;
    float col[3];      // Color::new64(...) = f64 -> f32
    double param;      // DiffuseMetal exponent (fuzz * 1000) / Dielectric refractive index
};

float f32(double x) { return (float)x; }

// scene.rs:157-191 balls_scene(seed, need_speed = false, checker = true)
std::vector<Ball> balls_scene(uint64_t seed) {
    std::vector<Ball> out;
    Ball g{};
    g.c[0] = 0.0; g.c[1] = -1000.0; g.c[2] = 0.0; g.r = 1000.0;
    g.kind = RS_MAT_LAMBERTIAN; g.checker = 1;
    out.push_back(g);
    SeedRandom rng(seed);
    // scene.rs:23-75 add_small_balls(bounce_height 0.9)
    const double bounce = 0.9;
    for (int a = -11; a < 11; ++a)
        for (int b = -11; b < 11; ++b) {
            Ball s{};
            s.c[0] = std::fma(0.9, rng.normal(), (double)a);
            s.c[1] = 0.2 + rng.normal() * bounce;
            s.c[2] = std::fma(0.9, rng.normal(), (double)b);
            s.r = 0.2;
            // avoid = (center.x, 0.2, 0.0); (center - avoid).length() with the fma dot (vec3.rs:152-161)
            const double dx = s.c[0] - s.c[0], dy = s.c[1] - 0.2, dz = s.c[2] - 0.0;
            const double len = std::sqrt(std::fma(dz, dz, std::fma(dx, dx, dy * dy)));
            const double ax = std::fabs(s.c[0]);
            const bool in_lane = (ax >= 0.0 && ax < 0.9) || (ax >= 3.1 && ax < 4.9);
            if (!(!in_lane || len >= 0.9)) continue;
            const double mat = rng.normal();
            if (mat < 0.8) {
                const double r = rng.normal(), gg = rng.normal(), bb = rng.normal();
                s.kind = RS_MAT_LAMBERTIAN;
                s.col[0] = f32(r); s.col[1] = f32(gg); s.col[2] = f32(bb);
            } else if (mat < 0.95) {
                const double r = rng.range(0.5, 1.0), gg = rng.range(0.5, 1.0), bb = rng.range(0.5, 1.0);
                s.col[0] = f32(r); s.col[1] = f32(gg); s.col[2] = f32(bb);
                const double fuzz = rng.range(0.0, 0.5);
                if (fuzz < 0.1) {
                    s.kind = RS_MAT_METAL;
                } else {
                    s.kind = RS_MAT_DIFFUSE_METAL;
                    s.param = fuzz * 1000.0;
                }
            } else {
                s.kind = RS_MAT_DIELECTRIC;
                s.col[0] = s.col[1] = s.col[2] = 1.0f;
                s.param = 1.5;
            }
            out.push_back(s);
        }
    // scene.rs:133-154 add_big_balls
    Ball b0{}; b0.c[1] = 1.0; b0.r = 1.0; b0.kind = RS_MAT_DIELECTRIC; b0.col[0] = b0.col[1] = b0.col[2] = 1.0f; b0.param = 1.5;
    Ball b1{}; b1.c[0] = -4.0; b1.c[1] = 1.0; b1.r = 1.0; b1.kind = RS_MAT_LAMBERTIAN;
    b1.col[0] = 0.4f; b1.col[1] = 0.2f; b1.col[2] = 0.1f;
    Ball b2{}; b2.c[0] = 4.0; b2.c[1] = 1.0; b2.r = 1.0; b2.kind = RS_MAT_METAL;
    b2.col[0] = 0.7f; b2.col[1] = 0.6f; b2.col[2] = 0.5f;
    out.push_back(b0); out.push_back(b1); out.push_back(b2);
    return out;
}

void solid(rs_texture_desc& t, float r, float g, float b) {
    std::memset(&t, 0, sizeof(t));
    t.kind = RS_TEX_SOLID;
    t.even[0] = t.odd[0] = r; t.even[1] = t.odd[1] = g; t.even[2] = t.odd[2] = b; t.even[3] = t.odd[3] = 1.0f;
    t.scale = 1.0;
}

}  // namespace

extern "C" {

// RFC 7539 check of the core: 16 state words in, `rounds` rounds, 16 words out
void orc_chacha_block(const uint32_t in[16], int rounds, uint32_t out[16]) { chacha_block(in, rounds, out); }

// the generated ball list, 12 doubles per sphere: cx cy cz r kind checker col_r col_g col_b param 0 0.
// Returns the sphere count (rows are written while count <= cap).
int orc_rtow_balls(uint64_t seed, double* out, int cap) {
    const std::vector<Ball> v = balls_scene(seed);
    for (size_t i = 0; i < v.size() && (int)i < cap; ++i) {
        double* o = out + 12 * i;
        const Ball& b = v[i];
        o[0] = b.c[0]; o[1] = b.c[1]; o[2] = b.c[2]; o[3] = b.r; o[4] = b.kind; o[5] = b.checker;
        o[6] = b.col[0]; o[7] = b.col[1]; o[8] = b.col[2]; o[9] = b.param; o[10] = 0.0; o[11] = 0.0;
    }
    return (int)v.size();
}

// examples/rtow_13_1.rs:15-46: balls_scene(seed) + the light sphere (300, 400, 100) r 12
// DiffuseLight(1, 0.9, 0.7) x1.5 in world and lights, gradient sky, time range 0..0 -- built straight
// into an oracle scene (one material per sphere, like the reference's per-sphere Arc).
int orc_rtow_scene(orc_scene* s, uint64_t seed) {
    const std::vector<Ball> v = balls_scene(seed);
    for (const Ball& b : v) {
        rs_material_desc d;
        std::memset(&d, 0, sizeof(d));
        d.kind = b.kind;
        d.refractive = 1.0; d.multiplier = 1.0; d.mix_p = 0.5; d.phong_exponent = 1;
        if (b.checker) {  // Checker::new(Color(0.3, 0.3, 0.3), Color(0.1, 0.1, 0.1), 10.0): odd, even
            std::memset(&d.texture, 0, sizeof(d.texture));
            d.texture.kind = RS_TEX_CHECKER;
            d.texture.odd[0] = d.texture.odd[1] = d.texture.odd[2] = 0.3f; d.texture.odd[3] = 1.0f;
            d.texture.even[0] = d.texture.even[1] = d.texture.even[2] = 0.1f; d.texture.even[3] = 1.0f;
            d.texture.scale = 10.0;
        } else {
            solid(d.texture, b.col[0], b.col[1], b.col[2]);
        }
        if (b.kind == RS_MAT_DIFFUSE_METAL) d.exponent = b.param;
        if (b.kind == RS_MAT_DIELECTRIC) { d.refractive = b.param; d.glass = 1; }
        int32_t m;
        int rc = orc_material(s, &d, &m);
        if (rc) return rc;
        uint32_t h;
        const double zero[3] = {0.0, 0.0, 0.0};
        if ((rc = orc_sphere(s, b.c, b.r, zero, m, &h))) return rc;
        if ((rc = orc_world_add(s, h))) return rc;
    }
    rs_material_desc L;
    std::memset(&L, 0, sizeof(L));
    L.kind = RS_MAT_DIFFUSE_LIGHT;
    solid(L.texture, 1.0f, 0.9f, 0.7f);
    L.refractive = 1.0; L.multiplier = 1.5; L.mix_p = 0.5; L.phong_exponent = 1;
    int32_t lm;
    int rc = orc_material(s, &L, &lm);
    if (rc) return rc;
    const double lc[3] = {300.0, 400.0, 100.0}, zero[3] = {0.0, 0.0, 0.0};
    uint32_t lh;
    if ((rc = orc_sphere(s, lc, 12.0, zero, lm, &lh))) return rc;
    if ((rc = orc_lights_add(s, lh))) return rc;
    if ((rc = orc_world_add(s, lh))) return rc;
    const float lo[3] = {0.3f, 0.4f, 0.5f}, hi[3] = {0.7f, 0.89f, 1.0f};
    if ((rc = orc_set_background(s, lo, hi))) return rc;
    return orc_set_time_range(s, 0.0, 0.0);
}

}  // extern "C"
