// libraysnail_host: scene assets of the host layer -- FastRng, Perlin tables, PNG images, OBJ meshes.
//
//   FastRng                 src/prelude/random.rs:109-145 (rand_xorshift 0.3.0 + rand_core 0.6.2)
//   FastRng::shuffle        rand 0.8.3 SliceRandom::shuffle + UniformInt<u32>::sample_single (restated)
//   Perlin::new             src/texture/noise.rs:44-66 (values Vec3::random_unit vec3.rs:91-96 / gen)
//   Image::open             src/texture/image.rs:24-31 (image 0.23.14 PNG decode -> get_pixel as RGB)
//   TriangleMesh::load      src/hittable/geometry/triangle_mesh.rs:166-276 over a tobj 4.0.2-compatible
//                           OBJ reader (LoadOptions{single_index, triangulate}, triangle_mesh.rs:175-183)
//
// The transcendental calls (random_unit's sin / cos, the mesh rotation's sin / cos) use the path's
// correctly rounded libm (include/rs_crmath.h), like the kernels.
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <tuple>

#include "raysnail.hpp"
#include "rs_crmath.h"

namespace raysnail {

namespace detail {
void set_error(const std::string& e);
}

// ---------------------------------------------------------------------------------- FastRng ----
FastRng::FastRng(uint64_t state) {
    uint32_t s[4];
    for (int i = 0; i < 4; ++i) {  // rand_core 0.6 seed_from_u64: PCG32 output words
        state = state * 6364136223846793005ULL + 11634580027462260723ULL;
        const uint32_t xs = (uint32_t)(((state >> 18) ^ state) >> 27);
        const uint32_t rot = (uint32_t)(state >> 59);
        s[i] = (xs >> rot) | (xs << ((32u - rot) & 31u));
    }
    if ((s[0] | s[1] | s[2] | s[3]) == 0u) s[0] = s[1] = s[2] = s[3] = 0x0BAD5EEDu;  // rand_xorshift from_seed
    x_ = s[0]; y_ = s[1]; z_ = s[2]; w_ = s[3];
}
uint32_t FastRng::next_u32() {
    const uint32_t t = x_ ^ (x_ << 11);
    x_ = y_; y_ = z_; z_ = w_;
    w_ = w_ ^ (w_ >> 19) ^ (t ^ (t >> 8));
    return w_;
}
uint64_t FastRng::next_u64() {
    const uint64_t lo = next_u32();
    const uint64_t hi = next_u32();
    return (hi << 32) | lo;
}
double FastRng::gen() { return (double)next_u64() / 18446744073709551616.0; }

// rand 0.8.3 UniformInt<u32>::sample_single(0, ubound): range = ubound, zone = (range << lz) - 1,
// accept v with lo(v * range) <= zone, return hi(v * range)
uint32_t FastRng::gen_index(uint32_t ubound) {
    const uint32_t range = ubound;
    if (range == 0) return next_u32();
    const uint32_t zone = (range << __builtin_clz(range)) - 1u;
    for (;;) {
        const uint32_t v = next_u32();
        const uint64_t m = (uint64_t)v * (uint64_t)range;
        if ((uint32_t)m <= zone) return (uint32_t)(m >> 32);
    }
}
void FastRng::shuffle(std::vector<uint32_t>& v) {
    for (size_t i = v.size(); i-- > 1;) std::swap(v[i], v[gen_index((uint32_t)(i + 1))]);
}

// ----------------------------------------------------------------------------------- Perlin ----
Perlin::Perlin(size_t point_count, bool vector, FastRng& rng) : d_(std::make_shared<PerlinData>()) {
    if (point_count == 0 || (point_count & (point_count - 1)) != 0)
        throw Error(RS_E_INVALID, "Perlin point_count must be a power of two (indices are masked, noise.rs:117)");
    PerlinData& d = *d_;
    d.point_count = (uint32_t)point_count;
    d.vector = vector;
    for (size_t i = 0; i < point_count; ++i) {
        if (vector) {  // Vec3::random_unit (vec3.rs:91-96)
            const double a = rng.range(0.0, 2.0 * 3.14159265358979323846);
            const double z = rng.range(-1.0, 1.0);
            const double r = std::sqrt(1.0 - z * z);
            double sa, ca;
            rs_cr::sincos_cr(a, &sa, &ca);
            d.values.push_back(r * ca);
            d.values.push_back(r * sa);
            d.values.push_back(z);
        } else {
            d.values.push_back(rng.gen());
        }
    }
    for (auto* perm : {&d.perm_x, &d.perm_y, &d.perm_z}) {
        perm->resize(point_count);
        for (size_t i = 0; i < point_count; ++i) (*perm)[i] = (uint32_t)i;
        rng.shuffle(*perm);
    }
}

// ------------------------------------------------------------------------------------ Image ----
Image::Image(uint32_t width, uint32_t height, std::vector<uint8_t> rgb) {
    if (width == 0 || height == 0 || rgb.size() != (size_t)width * height * 3)
        throw Error(RS_E_INVALID, "Image: width * height * 3 bytes of RGB expected");
    auto d = std::make_shared<ImageData>();
    d->width = width; d->height = height; d->rgb = std::move(rgb);
    d_ = d;
}

namespace {
uint32_t be32(const uint8_t* p) { return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3]; }
uint8_t paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    return (uint8_t)((pa <= pb && pa <= pc) ? a : pb <= pc ? b : c);
}
}  // namespace

Image Image::open(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw Error(RS_E_INVALID, "Image: cannot open " + path);
    std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    if (buf.size() < 8 || std::memcmp(buf.data(), sig, 8) != 0) throw Error(RS_E_INVALID, "Image: not a PNG file: " + path);
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte;
    size_t pos = 8;
    while (pos + 12 <= buf.size()) {
        const uint32_t len = be32(&buf[pos]);
        if (pos + 12 + (size_t)len > buf.size()) throw Error(RS_E_INVALID, "Image: truncated PNG chunk");
        const char* type = (const char*)&buf[pos + 4];
        const uint8_t* data = &buf[pos + 8];
        if (!std::memcmp(type, "IHDR", 4) && len >= 13) {
            w = be32(data); h = be32(data + 4); depth = data[8]; ctype = data[9]; interlace = data[12];
        } else if (!std::memcmp(type, "PLTE", 4)) {
            plte.assign(data, data + len);
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), data, data + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        pos += 12 + (size_t)len;
    }
    const int channels = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
    if (!w || !h || channels == 0) throw Error(RS_E_INVALID, "Image: bad PNG header");
    if (depth != 8 || interlace != 0)
        throw Error(RS_E_UNSUPPORTED, "Image: only 8-bit, non-interlaced PNGs are supported");
    // bound the header before sizing buffers from it (a crafted IHDR must fail, not overflow):
    // each side <= 2^24, decoded bytes (incl. one filter byte per row) <= 2^31, zlib sizes < 2^32
    if (w > (1u << 24) || h > (1u << 24)) throw Error(RS_E_INVALID, "Image: PNG dimensions too large");
    const uint64_t raw_bytes = ((uint64_t)w * (uint64_t)channels + 1) * (uint64_t)h;
    if (raw_bytes > (1ull << 31)) throw Error(RS_E_INVALID, "Image: PNG image too large (> 2 GiB decoded)");
    if (idat.size() > 0xFFFFFFFFull) throw Error(RS_E_INVALID, "Image: PNG image data too large");
    const size_t stride = (size_t)w * channels;
    std::vector<uint8_t> raw((stride + 1) * h);
    z_stream zs;
    std::memset(&zs, 0, sizeof(zs));
    if (inflateInit(&zs) != Z_OK) throw Error(RS_E_INVALID, "Image: zlib init failed");
    zs.next_in = idat.data(); zs.avail_in = (uInt)idat.size();
    zs.next_out = raw.data(); zs.avail_out = (uInt)raw.size();
    const int rc = inflate(&zs, Z_FINISH);
    inflateEnd(&zs);
    if (rc != Z_STREAM_END || zs.avail_out != 0) throw Error(RS_E_INVALID, "Image: corrupt PNG image data");
    // undo the per-row filters (PNG spec 9.2), bpp = channels bytes
    std::vector<uint8_t> px(stride * h);
    for (uint32_t y = 0; y < h; ++y) {
        const uint8_t ft = raw[y * (stride + 1)];
        const uint8_t* in = &raw[y * (stride + 1) + 1];
        uint8_t* out = &px[y * stride];
        const uint8_t* up = y ? &px[(y - 1) * stride] : nullptr;
        for (size_t i = 0; i < stride; ++i) {
            const int a = i >= (size_t)channels ? out[i - channels] : 0, b = up ? up[i] : 0,
                      c = (up && i >= (size_t)channels) ? up[i - channels] : 0;
            uint8_t v = in[i];
            switch (ft) {
            case 0: break;
            case 1: v = (uint8_t)(v + a); break;
            case 2: v = (uint8_t)(v + b); break;
            case 3: v = (uint8_t)(v + ((a + b) >> 1)); break;
            case 4: v = (uint8_t)(v + paeth(a, b, c)); break;
            default: throw Error(RS_E_INVALID, "Image: bad PNG filter type");
            }
            out[i] = v;
        }
    }
    // to RGB (DynamicImage::get_pixel -> Rgba<u8>; image.rs reads channels 0..2)
    std::vector<uint8_t> rgb((size_t)w * h * 3);
    for (size_t i = 0; i < (size_t)w * h; ++i) {
        const uint8_t* p = &px[i * channels];
        uint8_t r, g, b;
        if (ctype == 3) {
            if ((size_t)p[0] * 3 + 2 >= plte.size()) throw Error(RS_E_INVALID, "Image: palette index out of range");
            r = plte[p[0] * 3]; g = plte[p[0] * 3 + 1]; b = plte[p[0] * 3 + 2];
        } else if (channels <= 2) {
            r = g = b = p[0];
        } else {
            r = p[0]; g = p[1]; b = p[2];
        }
        rgb[3 * i] = r; rgb[3 * i + 1] = g; rgb[3 * i + 2] = b;
    }
    return Image(w, h, std::move(rgb));
}

// ------------------------------------------------------------------------------ OBJ / tobj ----
namespace {
struct ObjModel {
    std::vector<std::array<float, 3>> positions;   // per unified vertex
    std::vector<std::array<float, 3>> normals;     // per unified vertex (empty: the file has none)
    std::vector<uint32_t> indices;                 // 3 per triangle
};

// tobj 4.0.2 load_obj with single_index + triangulate: a model per o / g / usemtl group that has
// faces; each (v, vt, vn) index tuple of a model is one vertex; polygons become fans (a, b, c),
// (a, c, d), ...; negative indices count back from the current end
std::vector<ObjModel> read_obj(const std::string& filename) {
    std::ifstream f(filename);
    if (!f) throw Error(RS_E_INVALID, "TriangleMesh::load: cannot open " + filename);
    std::vector<std::array<float, 3>> v, vn;
    size_t n_vt = 0;
    std::vector<ObjModel> models;
    ObjModel cur;
    std::map<std::tuple<long, long, long>, uint32_t> ids;
    auto flush = [&] {
        if (!cur.indices.empty()) models.push_back(std::move(cur));
        cur = ObjModel();
        ids.clear();
    };
    auto parse_f = [&](const std::string& tok, const std::string& what) {
        char* e = nullptr;
        const float x = std::strtof(tok.c_str(), &e);
        if (e == tok.c_str()) throw Error(RS_E_INVALID, "TriangleMesh::load: bad " + what + " '" + tok + "'");
        return x;
    };
    auto index = [&](const std::string& s, size_t count) -> long {
        if (s.empty()) return -1;
        const long i = std::strtol(s.c_str(), nullptr, 10);
        const long r = i < 0 ? (long)count + i : i - 1;
        if (i == 0 || r < 0 || r >= (long)count) throw Error(RS_E_INVALID, "TriangleMesh::load: face index out of range");
        return r;
    };
    std::string line;
    while (std::getline(f, line)) {
        std::istringstream ls(line);
        std::string key;
        if (!(ls >> key) || key[0] == '#') continue;
        std::vector<std::string> t;
        for (std::string x; ls >> x;) t.push_back(x);
        if (key == "v") {
            if (t.size() < 3) throw Error(RS_E_INVALID, "TriangleMesh::load: v needs 3 coordinates");
            v.push_back({parse_f(t[0], "v"), parse_f(t[1], "v"), parse_f(t[2], "v")});
        } else if (key == "vn") {
            if (t.size() < 3) throw Error(RS_E_INVALID, "TriangleMesh::load: vn needs 3 coordinates");
            vn.push_back({parse_f(t[0], "vn"), parse_f(t[1], "vn"), parse_f(t[2], "vn")});
        } else if (key == "vt") {
            ++n_vt;
        } else if (key == "o" || key == "g" || key == "usemtl") {
            flush();
        } else if (key == "f") {
            if (t.size() < 3) continue;  // points / lines: no triangles
            std::vector<uint32_t> face;
            for (const std::string& tok : t) {
                std::string a[3];
                size_t k = 0;
                for (char c : tok) { if (c == '/') { if (++k > 2) break; } else a[k] += c; }
                const std::tuple<long, long, long> key3(index(a[0], v.size()), index(a[1], n_vt), index(a[2], vn.size()));
                auto it = ids.find(key3);
                if (it == ids.end()) {
                    const uint32_t id = (uint32_t)cur.positions.size();
                    cur.positions.push_back(v[std::get<0>(key3)]);
                    if (std::get<2>(key3) >= 0) cur.normals.push_back(vn[std::get<2>(key3)]);
                    it = ids.emplace(key3, id).first;
                }
                face.push_back(it->second);
            }
            for (size_t i = 2; i < face.size(); ++i) {
                cur.indices.push_back(face[0]);
                cur.indices.push_back(face[i - 1]);
                cur.indices.push_back(face[i]);
            }
        }
    }
    flush();
    return models;
}

// Vec3::rotate (vec3.rs:196-214)
void rotate(double p[3], int axis, double c, double s) {
    const double x = p[0], y = p[1], z = p[2];
    if (axis == 0) { p[1] = y * c - z * s; p[2] = y * s + z * c; }
    else if (axis == 1) { p[0] = x * c + z * s; p[2] = -x * s + z * c; }
    else { p[0] = x * c - y * s; p[1] = x * s + y * c; }
}
}  // namespace

std::shared_ptr<TriangleMesh> TriangleMesh::load(const std::string& filename, double scale, Vec3 offset,
                                                 double rotation_angle, int axis, MaterialRef material) {
    const std::vector<ObjModel> models = read_obj(filename);
    double sn, cs;
    rs_cr::sincos_cr(rotation_angle * (3.14159265358979323846 / 180.0), &sn, &cs);  // f64::to_radians
    std::vector<double> pos, nrm;
    for (const ObjModel& m : models) {
        const bool has_normals = !m.normals.empty();
        if (has_normals && m.normals.size() != m.positions.size())
            throw Error(RS_E_UNSUPPORTED, "TriangleMesh::load: some vertices of a model lack normals");
        // upstream sizes v_normal by the triangle count and indexes it by vertex (a panic when a
        // model has more vertices than triangles); here it has one entry per vertex
        std::vector<std::array<double, 3>> v_normal(m.positions.size(), {0.0, 0.0, 0.0});
        std::vector<std::array<double, 3>> rp(m.positions.size());
        for (size_t i = 0; i < m.positions.size(); ++i) {
            double p[3] = {(double)m.positions[i][0], (double)m.positions[i][1], (double)m.positions[i][2]};
            rotate(p, axis, cs, sn);
            rp[i] = {p[0], p[1], p[2]};
        }
        const size_t nt = m.indices.size() / 3;
        for (size_t t = 0; t < nt; ++t) {
            const uint32_t i0 = m.indices[3 * t], i1 = m.indices[3 * t + 1], i2 = m.indices[3 * t + 2];
            const auto &p0 = rp[i0], &p1 = rp[i1], &p2 = rp[i2];
            if (!has_normals) {  // face normal (p1 - p0) x (p2 - p0), unit (vec3.rs:182-194)
                const double a[3] = {p1[0] - p0[0], p1[1] - p0[1], p1[2] - p0[2]};
                const double b[3] = {p2[0] - p0[0], p2[1] - p0[1], p2[2] - p0[2]};
                const double c[3] = {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
                const double inv = 1.0 / std::sqrt(std::fma(c[2], c[2], std::fma(c[0], c[0], c[1] * c[1])));
                for (uint32_t k : {i0, i1, i2})
                    for (int j = 0; j < 3; ++j) v_normal[k][j] += c[j] * inv;
            }
            for (const auto* p : {&p0, &p1, &p2})
                for (int j = 0; j < 3; ++j) pos.push_back((*p)[j] * scale + (j == 0 ? offset.x : j == 1 ? offset.y : offset.z));
        }
        for (size_t t = 0; t < nt; ++t)
            for (int c = 0; c < 3; ++c) {
                const uint32_t k = m.indices[3 * t + c];
                double n[3];
                if (has_normals) {
                    n[0] = m.normals[k][0]; n[1] = m.normals[k][1]; n[2] = m.normals[k][2];
                    rotate(n, axis, cs, sn);
                } else {
                    const auto& q = v_normal[k];
                    const double inv = 1.0 / std::sqrt(std::fma(q[2], q[2], std::fma(q[0], q[0], q[1] * q[1])));
                    n[0] = q[0] * inv; n[1] = q[1] * inv; n[2] = q[2] * inv;
                }
                nrm.insert(nrm.end(), n, n + 3);
            }
    }
    return std::make_shared<TriangleMesh>(std::move(pos), std::move(nrm), std::move(material));
}

}  // namespace raysnail

using namespace raysnail;

namespace {
template <class F>
int guarded_assets(F&& f) {
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
template <class T>
T* malloc_copy(const std::vector<T>& v) {
    T* p = (T*)std::malloc(std::max<size_t>(1, v.size()) * sizeof(T));
    if (!p) throw std::bad_alloc();
    if (!v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
    return p;
}
}  // namespace

extern "C" int rsh_obj_load(const char* path, double scale, const double offset[3], double rotation_angle, int axis,
                            uint32_t* n, double** pos, double** nrm) {
    return guarded_assets([&] {
        if (!path || !offset || !n || !pos || !nrm) throw Error(RS_E_INVALID, "null argument");
        auto mesh = TriangleMesh::load(path, scale, Vec3{offset[0], offset[1], offset[2]}, rotation_angle, axis, nullptr);
        *n = (uint32_t)mesh->len();
        *pos = malloc_copy(mesh->positions());
        *nrm = malloc_copy(mesh->normals());
    });
}

extern "C" int rsh_perlin_tables(uint64_t seed, uint32_t point_count, int vector, double* values, uint32_t* perms) {
    return guarded_assets([&] {
        if (!values || !perms) throw Error(RS_E_INVALID, "null argument");
        FastRng rng(seed);
        Perlin p(point_count, vector != 0, rng);
        const PerlinData& d = *p.data();
        std::memcpy(values, d.values.data(), d.values.size() * sizeof(double));
        std::memcpy(perms, d.perm_x.data(), point_count * sizeof(uint32_t));
        std::memcpy(perms + point_count, d.perm_y.data(), point_count * sizeof(uint32_t));
        std::memcpy(perms + 2 * (size_t)point_count, d.perm_z.data(), point_count * sizeof(uint32_t));
    });
}

extern "C" int rsh_png_load(const char* path, uint32_t* width, uint32_t* height, uint8_t** rgb) {
    return guarded_assets([&] {
        if (!path || !width || !height || !rgb) throw Error(RS_E_INVALID, "null argument");
        Image im = Image::open(path);
        *width = im.data()->width;
        *height = im.data()->height;
        *rgb = malloc_copy(im.data()->rgb);
    });
}

extern "C" void rsh_free(void* p) { std::free(p); }
