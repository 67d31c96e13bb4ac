"""Scene assets and the §8(f)3-4 additions, CPU only: the PNG reader (Image::new), the OBJ reader
(TriangleMesh::load over a tobj-4.0.2-compatible parser), the Perlin tables (FastRng + rand 0.8's
shuffle), and independent Python restatements of noise.rs / BlinnPhongPdf / SpherePdf /
ConstantMedium's draw checked against the oracle's probes.

Pinning: no reference fixture covers these paths (the reference has one test, transform.rs:187-206;
its Perlin tables come from an OS-seeded FastRng, noise.rs:44-66 via scene.rs:424). The checks here
pin the oracle to restatements written independently in Python from the reference source; the
earth-map test decodes the reference's own examples/earth-map.png where the tree exists.
"""
import ctypes as C
import math
import os
import struct
import zlib

import numpy as np
import pytest

from raysnail_amd import _abi as A
from raysnail_amd import api, host_lib, scenes
from raysnail_amd.scenes import fma as _fma

EARTH = "/root/reference/examples/earth-map.png"


# ------------------------------------------------------------------------------------- PNG ----
def _png(path, pix, ctype, filters, palette=None):
    """Minimal PNG encoder: 8-bit, filter type per row from `filters` (independent of the C++ reader)."""
    h, w = pix.shape[:2]
    ch = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    raw = pix.reshape(h, w * ch).astype(np.int32)
    out = bytearray()
    for y in range(h):
        ft = filters[y % len(filters)]
        row, up = raw[y], raw[y - 1] if y else np.zeros(w * ch, np.int32)
        left = np.concatenate([np.zeros(ch, np.int32), row[:-ch]])
        ul = np.concatenate([np.zeros(ch, np.int32), up[:-ch]])
        if ft == 0:
            f = row
        elif ft == 1:
            f = row - left
        elif ft == 2:
            f = row - up
        elif ft == 3:
            f = row - (left + up) // 2
        else:
            p = left + up - ul
            pa, pb, pc = abs(p - left), abs(p - up), abs(p - ul)
            pred = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, up, ul))
            f = row - pred
        out.append(ft)
        out += bytes((f % 256).astype(np.uint8))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)
    data = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, ctype, 0, 0, 0))
    if palette is not None:
        data += chunk(b"PLTE", bytes(palette.astype(np.uint8).reshape(-1)))
    comp = zlib.compress(bytes(out), 6)
    data += chunk(b"IDAT", comp[: len(comp) // 2]) + chunk(b"IDAT", comp[len(comp) // 2:]) + chunk(b"IEND", b"")
    open(path, "wb").write(data)


@pytest.mark.parametrize("ctype", [0, 2, 3, 4, 6])
def test_png_reader_color_types_and_filters(tmp_path, ctype):
    rng = np.random.default_rng(ctype)
    h, w = 13, 17
    ch = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    pix = rng.integers(0, 256, (h, w, ch), dtype=np.uint8)
    pal = None
    if ctype == 3:
        pal = rng.integers(0, 256, (256, 3), dtype=np.uint8)
    path = str(tmp_path / f"t{ctype}.png")
    _png(path, pix, ctype, [0, 1, 2, 3, 4], pal)
    got = host_lib.png_load(path)
    if ctype == 3:
        want = pal[pix[..., 0]]
    elif ch <= 2:
        want = np.repeat(pix[..., :1], 3, axis=2)
    else:
        want = pix[..., :3]
    assert np.array_equal(got, want)


def test_png_reader_roundtrips_own_writer(tmp_path):
    rgba = np.random.default_rng(1).random((20, 30, 4)).astype(np.float32)
    host_lib.write_png(str(tmp_path / "w.png"), rgba)
    got = host_lib.png_load(str(tmp_path / "w.png"))
    want = (np.clip(rgba[..., :3], 0, 1) * 255.5).astype(np.uint8)  # raysnail.rs:437-439
    assert np.array_equal(got, want)


def test_png_reader_rejects_bad_files(tmp_path):
    p = tmp_path / "x.png"
    p.write_bytes(b"not a png")
    with pytest.raises(host_lib.HostError):
        host_lib.png_load(str(p))
    with pytest.raises(host_lib.HostError):
        host_lib.png_load(str(tmp_path / "missing.png"))


@pytest.mark.parametrize("w,h", [(2 ** 31, 2 ** 31), (1 << 25, 1), (1 << 24, 1 << 24), (0, 5)])
def test_png_reader_rejects_oversized_headers(tmp_path, w, h):
    """A crafted IHDR (sizes whose byte counts overflow 32/64-bit products) fails cleanly before any
    buffer is sized from it; the reference's image crate fails safely on these too."""
    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)
    data = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 6, 0, 0, 0))
    data += chunk(b"IDAT", zlib.compress(b"\x00" * 64)) + chunk(b"IEND", b"")
    p = tmp_path / "big.png"
    p.write_bytes(data)
    with pytest.raises(host_lib.HostError):
        host_lib.png_load(str(p))


@pytest.mark.skipif(not os.path.exists(EARTH), reason="reference tree absent")
def test_png_reader_on_reference_earth_map():
    """examples/earth-map.png (1920x960 RGB): the C++ reader against zlib + numpy unfiltering."""
    data = open(EARTH, "rb").read()
    pos, idat, hdr = 8, b"", None
    while pos < len(data):
        n = struct.unpack(">I", data[pos:pos + 4])[0]
        t = data[pos + 4:pos + 8]
        if t == b"IHDR":
            hdr = struct.unpack(">IIBBBBB", data[pos + 8:pos + 21])
        elif t == b"IDAT":
            idat += data[pos + 8:pos + 8 + n]
        pos += 12 + n
    w, h, depth, ctype = hdr[:4]
    assert (depth, ctype) == (8, 2)
    raw = np.frombuffer(zlib.decompress(idat), np.uint8).reshape(h, 1 + 3 * w)
    img = np.zeros((h, 3 * w), np.int32)
    for y in range(h):
        ft, row = raw[y, 0], raw[y, 1:].astype(np.int32)
        up = img[y - 1] if y else np.zeros(3 * w, np.int32)
        cur = np.zeros(3 * w, np.int32)
        for x in range(3 * w):  # sequential (Sub / Average / Paeth depend on the left neighbour)
            a = cur[x - 3] if x >= 3 else 0
            b = up[x]
            c = up[x - 3] if x >= 3 else 0
            if ft == 0:
                v = row[x]
            elif ft == 1:
                v = row[x] + a
            elif ft == 2:
                v = row[x] + b
            elif ft == 3:
                v = row[x] + (a + b) // 2
            else:
                p = a + b - c
                pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
                v = row[x] + (a if pa <= pb and pa <= pc else b if pb <= pc else c)
            cur[x] = v & 255
        img[y] = cur
        if y == 40:  # 41 full rows through the pure-Python unfilter is enough of a check
            break
    got = host_lib.png_load(EARTH)
    assert got.shape == (h, w, 3)
    assert np.array_equal(got[:41].reshape(41, 3 * w), img[:41])


# ------------------------------------------------------------------------------------- OBJ ----
def _rot(p, axis, c, s):
    x, y, z = p
    if axis == 0:
        return (x, y * c - z * s, y * s + z * c)
    if axis == 1:
        return (x * c + z * s, y, -x * s + z * c)
    return (x * c - y * s, x * s + y * c, z)


def _f32(x):
    return float(np.float32(x))


def _obj_restated(text, scale, offset, angle, axis):
    """triangle_mesh.rs:166-276 over tobj (single_index, triangulate), written from the reference
    independently of raysnail_amd/host/assets.cpp; sin / cos taken from the library's own
    correctly rounded routine through a 1-triangle probe is avoided by passing angle 0 or 90/180."""
    v, vn, nvt = [], [], 0
    models, cur, ids = [], {"pos": [], "nrm": [], "idx": []}, {}

    def flush():
        nonlocal cur, ids
        if cur["idx"]:
            models.append(cur)
        cur, ids = {"pos": [], "nrm": [], "idx": []}, {}

    for line in text.splitlines():
        t = line.split()
        if not t or t[0].startswith("#"):
            continue
        if t[0] == "v":
            v.append(tuple(_f32(x) for x in t[1:4]))
        elif t[0] == "vn":
            vn.append(tuple(_f32(x) for x in t[1:4]))
        elif t[0] == "vt":
            nvt += 1
        elif t[0] in ("o", "g", "usemtl"):
            flush()
        elif t[0] == "f" and len(t) >= 4:
            face = []
            for tok in t[1:]:
                parts = (tok.split("/") + ["", ""])[:3]

                def ix(sv, n):
                    if sv == "":
                        return -1
                    i = int(sv)
                    return n + i if i < 0 else i - 1
                key = (ix(parts[0], len(v)), ix(parts[1], nvt), ix(parts[2], len(vn)))
                if key not in ids:
                    ids[key] = len(cur["pos"])
                    cur["pos"].append(v[key[0]])
                    if key[2] >= 0:
                        cur["nrm"].append(vn[key[2]])
                face.append(ids[key])
            for i in range(2, len(face)):
                cur["idx"] += [face[0], face[i - 1], face[i]]
    flush()
    c = math.cos(math.radians(angle)) if angle % 90 else round(math.cos(math.radians(angle)))
    s = math.sin(math.radians(angle)) if angle % 90 else round(math.sin(math.radians(angle)))
    P, N = [], []
    for m in models:
        rp = [_rot(p, axis, c, s) for p in m["pos"]]
        vnorm = [[0.0, 0.0, 0.0] for _ in rp]
        idx = m["idx"]
        for t in range(len(idx) // 3):
            i0, i1, i2 = idx[3 * t:3 * t + 3]
            p0, p1, p2 = rp[i0], rp[i1], rp[i2]
            if not m["nrm"]:
                a = [p1[k] - p0[k] for k in range(3)]
                b = [p2[k] - p0[k] for k in range(3)]
                cr = [a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]]
                inv = 1.0 / math.sqrt(_fma(cr[2], cr[2], _fma(cr[0], cr[0], cr[1] * cr[1])))
                for k in (i0, i1, i2):
                    for j in range(3):
                        vnorm[k][j] += cr[j] * inv
            P.append([q[j] * scale + offset[j] for q in (p0, p1, p2) for j in range(3)])
        for t in range(len(idx) // 3):
            row = []
            for k in idx[3 * t:3 * t + 3]:
                if m["nrm"]:
                    row += list(_rot(m["nrm"][k], axis, c, s))
                else:
                    q = vnorm[k]
                    inv = 1.0 / math.sqrt(_fma(q[2], q[2], _fma(q[0], q[0], q[1] * q[1])))
                    row += [q[0] * inv, q[1] * inv, q[2] * inv]
            N.append(row)
    return np.array(P).reshape(-1, 9), np.array(N).reshape(-1, 9)


OBJ_QUADS = """# a unit cube of quads, no normals, two groups, negative indices in the second
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v 0 0 1
v 1 0 1
v 1 1 1
v 0 1 1
vt 0 0
vt 1 0
vt 1 1
g front
f 1/1 2/2 3/3 4/1
f 5 8 7 6
f 1 5 6 2
g back
f -8 -4 -1 -5
f -7 -6 -2 -3
f -5 -1 -2 -6
"""

OBJ_NORMALS = """o tetra
v 0.1 0.2 0.3
v 1.5 0.25 -0.5
v 0.3 1.7 0.4
v -0.2 0.1 1.9
vn 0.577 0.577 0.577
vn -1 0 0
vn 0 -1 0.0
vn 0 0 -1
f 1//4 3//4 2//4
f 1//2 4//2 3//2
f 1//3 2//3 4//3
f 2//1 3//1 4//1
usemtl other
f 1//1 2//2 3//3 4//4
"""


@pytest.mark.parametrize("text,scale,offset,angle,axis", [
    (OBJ_QUADS, 1.0, (0.0, 0.0, 0.0), 0.0, 1),
    (OBJ_QUADS, 0.2, (1.0, -2.0, 0.5), 90.0, 1),
    (OBJ_NORMALS, 2.5, (0.0, 1.0, 0.0), 180.0, 0),
    (OBJ_NORMALS, 1.0, (0.0, 0.0, 0.0), 90.0, 2),
])
def test_obj_reader_matches_restatement(tmp_path, text, scale, offset, angle, axis):
    path = tmp_path / "m.obj"
    path.write_text(text)
    pos, nrm = host_lib.obj_load(str(path), scale, offset, angle, axis)
    P, N = _obj_restated(text, scale, offset, angle, axis)
    assert pos.shape == P.shape and nrm.shape == N.shape
    # angles that are multiples of 90 degrees: the library's correctly rounded sin / cos of
    # (angle * pi / 180) differ from the exact 0 / 1 by < 1e-16, so compare with a tight bound
    assert np.allclose(pos, P, rtol=0, atol=1e-12) and np.allclose(nrm, N, rtol=0, atol=1e-12)
    if angle == 0.0:
        assert np.array_equal(pos, P) and np.array_equal(nrm, N)


def test_obj_reader_errors(tmp_path):
    p = tmp_path / "bad.obj"
    p.write_text("v 0 0 0\nf 1 2 3\n")
    with pytest.raises(host_lib.HostError):
        host_lib.obj_load(str(p), 1.0, (0, 0, 0), 0.0, 1)
    with pytest.raises(host_lib.HostError):
        host_lib.obj_load(str(tmp_path / "missing.obj"), 1.0, (0, 0, 0), 0.0, 1)


# ---------------------------------------------------------------------------------- Perlin ----
def _fastrng(seed):
    words = scenes.pcg32_seed_words(seed, 4)
    st = list(words)

    def u32():
        x, y, z, w = st
        t = (x ^ (x << 11)) & 0xFFFFFFFF
        w2 = (w ^ (w >> 19) ^ (t ^ (t >> 8))) & 0xFFFFFFFF
        st[:] = [y, z, w, w2]
        return w2
    return u32


def _perlin_tables_restated(seed, n, vector):
    """noise.rs:44-66 + rand 0.8.3 shuffle (gen_range(0..i+1) via UniformInt<u32>::sample_single)."""
    u32 = _fastrng(seed)

    def gen():
        lo = u32()
        hi = u32()
        return float((hi << 32) | lo) / 18446744073709551616.0

    vals = []
    for _ in range(n):
        if vector:
            a = 0.0 + gen() * (2.0 * math.pi - 0.0)
            z = -1.0 + gen() * (1.0 - -1.0)
            r = math.sqrt(1.0 - z * z)
            vals.append((r, a, z))
        else:
            vals.append(gen())
    perms = []
    for _ in range(3):
        p = list(range(n))
        for i in range(n - 1, 0, -1):
            rng_ = i + 1
            zone = ((rng_ << (32 - rng_.bit_length())) & 0xFFFFFFFF) - 1
            while True:
                m = u32() * rng_
                if (m & 0xFFFFFFFF) <= zone:
                    j = m >> 32
                    break
            p[i], p[j] = p[j], p[i]
        perms += p
    return vals, perms


@pytest.mark.parametrize("n,vector", [(256, True), (64, False), (2, False)])
def test_perlin_tables_restated(n, vector):
    values, perms = host_lib.perlin_tables(17, n, vector)
    vals, P = _perlin_tables_restated(17, n, vector)
    assert perms.tolist() == P
    if vector:
        v = values.reshape(-1, 3)
        for (r, a, z), got in zip(vals, v):
            assert got[2] == z
            # r cos a / r sin a with correctly rounded sin / cos (libm may differ by an ulp)
            assert abs(got[0] - r * math.cos(a)) <= 1e-15 and abs(got[1] - r * math.sin(a)) <= 1e-15
    else:
        assert values.tolist() == vals


def _noise_restated(t: api.Perlin, p):
    """noise.rs:111-211 for one point (Python restatement)."""
    n = t.point_count
    mask = n - 1
    vals = t.values.reshape(-1, 3) if t.vector else t.values
    px, py, pz = t.perms[:n], t.perms[n:2 * n], t.perms[2 * n:]

    def noise(q):
        if t._smooth == A.RS_SMOOTH_NONE:
            i, j, k = (int(4.0 * c) & mask for c in q)
            idx = px[i] ^ py[j] ^ pz[k]
            return float(vals[idx][0] if t.vector else vals[idx])
        i, j, k = (math.floor(c) for c in q)
        u, v, w = q[0] - i, q[1] - j, q[2] - k
        uu, vv, ww = u, v, w
        if t._smooth == A.RS_SMOOTH_HERMITE:
            uu, vv, ww = u * u * (3.0 - 2.0 * u), v * v * (3.0 - 2.0 * v), w * w * (3.0 - 2.0 * w)
        si = 0.0
        for a in range(2):
            sj = 0.0
            for b in range(2):
                sk = 0.0
                for c in range(2):
                    idx = px[(i + a) & mask] ^ py[(j + b) & mask] ^ pz[(k + c) & mask]
                    if t.vector:
                        g = vals[idx]
                        wx, wy, wz = u - a, v - b, w - c
                        val = _fma(g[2], wz, _fma(g[0], wx, g[1] * wy))
                    else:
                        val = float(vals[idx])
                    sk = sk + _fma(a, uu, (1 - a) * (1.0 - uu)) * _fma(b, vv, (1 - b) * (1.0 - vv)) \
                        * _fma(c, ww, (1 - c) * (1.0 - ww)) * val
                sj = sj + sk
            si = si + sj
        return si

    def turb(q, d):
        acc, weight = 0.0, 1.0
        for _ in range(d):
            acc = acc + weight * noise(q)
            weight *= 0.5
            q = (q[0] * 2.0, q[1] * 2.0, q[2] * 2.0)
        return abs(acc)

    if t._type == A.RS_PERLIN_TURBULENCE:
        return turb(p, t._depth)
    if t._type == A.RS_PERLIN_MARBLE:
        return None  # sin: checked in the GPU parity tests (correctly rounded on both sides)
    r = noise((t._scale * p[0], t._scale * p[1], t._scale * p[2]))
    return 0.5 * (r + 1.0) if t.vector else r


def _scatter_probe(oracle_lib, mat, ray, hit, seed):
    """orc_scatter on a one-material oracle scene: [ok, skip, has_ray, rgb, ray o, d, pdf dir, pdf value]."""
    from oracle.binding import OracleScene
    w = api.World(api.HittableList().add(api.Sphere((0, 0, 0), 1.0, mat)), api.HittableList().add(
        api.Sphere((0, 5, 0), 1.0, api.DiffuseLight(api.Color(1, 1, 1)))))
    orc = OracleScene(w)
    out = (C.c_double * 16)()
    assert oracle_lib.orc_scatter(orc.h, 0, (C.c_double * 7)(*ray), (C.c_double * 8)(*hit), seed, out) == 0
    return list(out)


@pytest.mark.parametrize("tex", [
    lambda: api.Perlin(256, True, 3).scale(0.7),
    lambda: api.Perlin(64, False, 5).smooth(api.SmoothType.None_).scale(3.0),
    lambda: api.Perlin(32, False, 4).smooth(api.SmoothType.LinearInterpolate).scale(5.0),
    lambda: api.Perlin(128, True, 9).turbulence(7),
])
def test_oracle_perlin_matches_restatement(oracle_lib, tex):
    t = tex()
    rng = np.random.default_rng(2)
    for _ in range(50):
        p = tuple(rng.uniform(-20, 20, 3))
        out = _scatter_probe(oracle_lib, api.Lambertian(t), (0, 0, 5, 0, 0, -1, 0), (*p, 0, 0, 1, 1.0, 1), 1)
        want = np.float32(_noise_restated(t, p))
        assert out[3] == out[4] == out[5] == float(want), (p, out[3], want)


def test_oracle_blinn_phong_and_sphere_pdf(oracle_lib):
    """BlinnPhongPdf (pdf.rs:144-212) and SpherePdf (pdf.rs:215-238) values at the generated direction."""
    d = np.array([0.3, -0.8, 0.2]); d /= np.linalg.norm(d)
    n = np.array([0.1, 0.95, 0.05]); n /= np.linalg.norm(n)
    for seed in range(1, 40):
        out = _scatter_probe(oracle_lib, api.BlinnPhong(0.5, 4.0, api.Color(0.9, 0.5, 0.1)),
                             (0, 2, 0, *d, 0), (0, 1, 0, *n, 1.0, 1), seed)
        assert out[:3] == [1.0, 0.0, 0.0]
        g = np.array(out[12:15])
        rn = -d + g
        rn = rn * (1.0 / math.sqrt(_fma(rn[2], rn[2], _fma(rn[0], rn[0], rn[1] * rn[1]))))
        dot = lambda a, b: _fma(a[2], b[2], _fma(a[0], b[0], a[1] * b[1]))
        cos = dot(g, n)
        cs = max(dot(rn, n), 0.0)
        npdf = (4.0 + 1.0) / (2.0 * math.pi) * cs ** 4.0
        want = max(cos / math.pi, 0.0) * (1.0 - 0.5) + npdf / (4.0 * dot(d * -1.0, rn)) * 0.5
        assert abs(out[15] - want) <= 1e-15 * max(1.0, abs(want)), (seed, out[15], want)
        iso = _scatter_probe(oracle_lib, api.Isotropic(api.Color(0.2, 0.4, 0.9)), (0, 2, 0, *d, 0),
                             (0, 1, 0, 1, 0, 0, 1.0, 0), seed)
        assert iso[15] == 1.0 / (4.0 * math.pi) and abs(np.linalg.norm(iso[12:15]) - 1.0) < 1e-12
        assert iso[3:6] == [float(np.float32(0.2)), float(np.float32(0.4)), float(np.float32(0.9))]


def test_medium_uniform_hash(hip_lib):
    """The determinism contract's ConstantMedium draw (rs_medium_uniform) restated."""
    M = 0xFFFFFFFFFFFFFFFF

    def sm(x):
        z = (x + 0x9E3779B97F4A7C15) & M
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M
        return z ^ (z >> 31)
    for st, h in [((1, 2, 3, 4), 0), ((0xDEADBEEF, 7, 0, 0xFFFFFFFF), 12345)]:
        key = sm(((st[1] << 32) | st[0]) ^ sm((st[3] << 32) | st[2]))
        want = float(sm(key ^ sm((0x6D656469756D2121 + h) & M))) * 2.0 ** -64
        assert hip_lib.rs_medium_uniform((C.c_uint32 * 4)(*st), h) == want


def test_new_scenes_realise_on_oracle(oracle_lib):
    """cornell_smoke / all_feature_scene / materials_scene build and render finite frames on the oracle."""
    from oracle.binding import OracleScene
    for cam, world in (scenes.cornell_smoke(24, 24), scenes.all_feature_scene(24, 24), scenes.materials_scene(32, 20)):
        photo = cam.take_photo().samples(4).depth(8).seed(1)
        img, st = OracleScene(world).render(cam.desc, photo.settings(), threads=4)
        assert np.isfinite(img).all() and st.segments > 0


def test_invalid_texture_and_medium_inputs(hip_lib):
    lib = hip_lib
    s = C.c_void_p()
    assert lib.rs_scene_create(C.byref(s)) == 0
    d = A.rs_material_desc()
    d.kind, d.refractive = A.RS_MAT_LAMBERTIAN, 1.0
    d.texture.kind, d.texture.data = A.RS_TEX_PERLIN, 3
    mid = C.c_int32()
    assert lib.rs_material(s, C.byref(d), C.byref(mid)) == A.RS_E_INVALID  # unknown perlin id
    pd = A.rs_perlin_desc()
    pd.point_count = 3  # not a power of two
    vals = (C.c_double * 9)()
    perm = (C.c_uint32 * 3)(0, 1, 2)
    pd.values, pd.perm_x, pd.perm_y, pd.perm_z = vals, perm, perm, perm
    assert lib.rs_perlin(s, C.byref(pd), C.byref(mid)) == A.RS_E_INVALID
    out = C.c_uint32()
    assert lib.rs_constant_medium(s, 99, (C.c_float * 4)(1, 1, 1, 1), 0.1, C.byref(out)) == A.RS_E_INVALID
    lib.rs_scene_destroy(s)
