"""Scene builders for the BASELINE configs (host side, run once per scene).

* RTIOW "balls" scene (examples/common/scene.rs:23-191) as used by examples/rtow_13_1.rs:15-52.
  Its layout depends on rand 0.8.3's StdRng (ChaCha12 from rand_chacha 0.3.0, seeded through
  rand_core 0.6's seed_from_u64) and UniformFloat sampling; those crates are not in the container,
  so they are restated below from their published algorithms. The ChaCha block function is pinned
  by the RFC 7539 test vector (tests/test_scenes.py); the buffering / float sampling is not pinned
  by any reference fixture ("raysnail-seed-7 (unverified restatement)").
* sdl/example.sdl and sdl/quadric.sdl hand-translated with the CLI's conventions
  (src/bin/raysnail.rs:340-367: aperture 0.01, focus 10, light spheres r=12 x1.7, gradient background).
* Cornell box (examples/common/scene.rs:211-334), with smoke (ConstantMedium boxes).
* all_feature_scene (examples/common/scene.rs:336-469): boxes, moving sphere, glass / metal,
  media, an Image-textured sphere (examples/earth-map.png when the reference tree is present, a
  synthetic image of the same size otherwise) and a Perlin sphere.
* materials_scene: a small build-owned scene exercising BlinnPhong, every Perlin variant, an Image
  texture, an Isotropic medium and a Difference (GPU-vs-oracle parity fixture).
"""
from __future__ import annotations

import math
from fractions import Fraction
from typing import List, Tuple

import numpy as np

import os

from .api import (AARect, AARectMetrics, BVH, BlinnPhong, Box, CameraBuilder, Checker, Color, ConstantMedium,
                  Dielectric, Difference, DiffuseLight, DiffuseMetal, Glass, Gradient, HittableList, Image,
                  Intersection, Lambertian, Metal, Perlin, Point3, Quadric, SmoothType, Sphere, TfFacade,
                  Transform, TransformStack, TriangleMesh, World)

M32 = 0xFFFFFFFF
M64 = 0xFFFFFFFFFFFFFFFF


def fma(a: float, b: float, c: float) -> float:
    """Correctly rounded a*b+c (f64::mul_add)."""
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def _rotl(x, n):
    return ((x << n) | (x >> (32 - n))) & M32


def chacha_block(key: List[int], counter: int, nonce: Tuple[int, int, int], rounds: int) -> List[int]:
    """ChaCha block function (RFC 7539 layout: constants, 8 key words, 32-bit counter, 3 nonce
    words). rand_chacha uses a 64-bit counter in words 12-13 and a 64-bit stream id in 14-15; with
    stream 0 and counters < 2^32 the two layouts coincide (word 13 = counter high = nonce[0] = 0)."""
    s = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + list(key) + [counter & M32] + list(nonce)
    x = list(s)

    def qr(a, b, c, d):
        x[a] = (x[a] + x[b]) & M32; x[d] = _rotl(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & M32; x[b] = _rotl(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & M32; x[d] = _rotl(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & M32; x[b] = _rotl(x[b] ^ x[c], 7)

    for _ in range(rounds // 2):
        qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
        qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
    return [(x[i] + s[i]) & M32 for i in range(16)]


def pcg32_seed_words(state: int, n_words: int) -> List[int]:
    """rand_core 0.6 SeedableRng::seed_from_u64: PCG32 output words (little-endian into the seed)."""
    out = []
    for _ in range(n_words):
        state = (state * 6364136223846793005 + 11634580027462260723) & M64
        xorshifted = (((state >> 18) ^ state) >> 27) & M32
        rot = state >> 59
        out.append(((xorshifted >> rot) | (xorshifted << ((32 - rot) & 31))) & M32)
    return out


class StdRng:
    """rand 0.8.3 StdRng = rand_chacha 0.3.0 ChaCha12Rng behind rand_core's BlockRng (64-word buffer
    = 4 consecutive ChaCha blocks)."""

    def __init__(self, seed_u64: int):
        self.key = pcg32_seed_words(seed_u64, 8)
        self.counter = 0
        self.results = [0] * 64
        self.index = 64

    def _generate(self):
        res = []
        for i in range(4):
            res += chacha_block(self.key, self.counter + i, (0, 0, 0), 12)
        self.counter += 4
        self.results = res

    def next_u32(self) -> int:
        if self.index >= 64:
            self._generate()
            self.index = 0
        v = self.results[self.index]
        self.index += 1
        return v

    def next_u64(self) -> int:  # rand_core BlockRng::next_u64
        if self.index < 63:
            lo, hi = self.results[self.index], self.results[self.index + 1]
            self.index += 2
            return (hi << 32) | lo
        if self.index >= 64:
            self._generate()
            self.index = 2
            return (self.results[1] << 32) | self.results[0]
        x = self.results[63]
        self._generate()
        self.index = 1
        return (self.results[0] << 32) | x


def _f64_from_bits(b: int) -> float:
    return float(np.array([b], dtype=np.uint64).view(np.float64)[0])


def _value0_1(rng: StdRng) -> float:
    # (u64 >> 12).into_float_with_exponent(0) - 1.0
    return _f64_from_bits((1023 << 52) | (rng.next_u64() >> 12)) - 1.0


def _next_down_pos(x: float) -> float:
    b = int(np.array([x], dtype=np.float64).view(np.uint64)[0])
    return _f64_from_bits(b - 1)


class SeedRandom:
    """src/prelude/random.rs:77-106 over StdRng; gen_range restated from rand 0.8.3 UniformFloat."""

    def __init__(self, seed: int):
        self.rng = StdRng(seed)

    def normal(self) -> float:
        # gen_range(0.0..=1.0): UniformFloat::new_inclusive(0, 1) then sample
        max_rand = 1.0 - 2.0 ** -52
        scale = (1.0 - 0.0) / max_rand
        while scale * max_rand + 0.0 > 1.0:
            scale = _next_down_pos(scale)
        return _value0_1(self.rng) * scale + 0.0

    def range(self, low: float, high: float) -> float:
        # gen_range(low..high): UniformFloat::sample_single
        scale = high - low
        while True:
            res = _value0_1(self.rng) * scale + low
            if res < high:
                return res
            scale = _next_down_pos(scale)


def _length(v):
    x, y, z = v
    return math.sqrt(fma(z, z, fma(x, x, y * y)))


def add_small_balls(world: HittableList, rng: SeedRandom, bounce_height: float):
    """examples/common/scene.rs:23-75 (need_speed = false)."""
    small_ball_radius = 0.2
    for a in range(-11, 11):
        for b in range(-11, 11):
            cx = fma(0.9, rng.normal(), float(a))
            cy = 0.2 + rng.normal() * bounce_height
            cz = fma(0.9, rng.normal(), float(b))
            center = (cx, cy, cz)
            ax = abs(cx)
            diff = (0.0, cy - 0.2, cz - 0.0)
            if not ((0.0 <= ax < 0.9) or (3.1 <= ax < 4.9)) or _length(diff) >= 0.9:
                mat = rng.normal()
                if mat < 0.8:
                    r, g, bb = rng.normal(), rng.normal(), rng.normal()
                    col = Color(float(np.float32(r)), float(np.float32(g)), float(np.float32(bb)), 1.0)
                    world.add(Sphere(center, small_ball_radius, Lambertian(col)))
                elif mat < 0.95:
                    r, g, bb = rng.range(0.5, 1.0), rng.range(0.5, 1.0), rng.range(0.5, 1.0)
                    col = Color(float(np.float32(r)), float(np.float32(g)), float(np.float32(bb)), 1.0)
                    fuzz = rng.range(0.0, 0.5)
                    if fuzz < 0.1:
                        world.add(Sphere(center, small_ball_radius, Metal(col)))
                    else:
                        world.add(Sphere(center, small_ball_radius, DiffuseMetal(fuzz * 1000.0, col)))
                else:
                    world.add(Sphere(center, small_ball_radius,
                                     Dielectric(Color(1.0, 1.0, 1.0, 1.0), 1.5).reflect_curve(Glass())))


def add_big_balls(world: HittableList):
    """examples/common/scene.rs:133-154"""
    world.add(Sphere((0.0, 1.0, 0.0), 1.0, Dielectric(Color(1.0, 1.0, 1.0, 1.0), 1.5).reflect_curve(Glass())))
    world.add(Sphere((-4.0, 1.0, 0.0), 1.0, Lambertian(Color(0.4, 0.2, 0.1, 1.0))))
    world.add(Sphere((4.0, 1.0, 0.0), 1.0, Metal(Color(0.7, 0.6, 0.5, 1.0))))


def f32(x: float) -> float:
    return float(np.float32(x))


def C32(r, g, b, a=1.0) -> Color:
    """Color::new takes f32 literals: round the decimal literal to f32 like rustc does."""
    return Color(f32(r), f32(g), f32(b), f32(a))


def balls_scene(seed: int = 7, checker: bool = True) -> HittableList:
    """examples/common/scene.rs:157-191 (need_speed = false)."""
    lst = HittableList()
    if checker:
        lst.add(Sphere((0.0, -1000.0, 0.0), 1000.0,
                       Lambertian(Checker(C32(0.3, 0.3, 0.3), C32(0.1, 0.1, 0.1), 10.0))))
    else:
        lst.add(Sphere((0.0, -1000.0, 0.0), 1000.0, Lambertian(C32(0.5, 0.5, 0.5))))
    rng = SeedRandom(seed)
    add_small_balls(lst, rng, 0.9)
    add_big_balls(lst)
    return lst


def balls_scene_camera() -> CameraBuilder:
    """examples/common/scene.rs:194-208 (need_shutter_speed = false)."""
    return CameraBuilder().look_from(Point3(13.0, 2.0, 3.0)).look_at(Point3(0.0, 0.0, 0.0)).fov(20.0) \
        .aperture(0.02).focus(10.0)


def _finish_balls(width: int, height: int, seed: int):
    """examples/rtow_13_1.rs:15-46: light sphere in both lists, gradient background."""
    world = balls_scene(seed, True)
    lights = HittableList()
    rs = Sphere((300.0, 400.0, 100.0), 12.0, DiffuseLight(C32(1.0, 0.9, 0.7)).multiplier(1.5))
    lights.add(rs)
    world.add(rs)
    camera = balls_scene_camera().width(width).height(height).build()
    w = World(world, lights, Gradient(C32(0.3, 0.4, 0.5), C32(0.7, 0.89, 1.0)), (0.0, camera.shutter_speed))
    return camera, w


def rtow_13_1(width: int = 800, height: int = 500, seed: int = 7):
    """Returns (camera, world, samples=122, depth=8) exactly as examples/rtow_13_1.rs."""
    camera, world = _finish_balls(width, height, seed)
    return camera, world, 122, 8


def _cli_world(hittables: HittableList, lights_at, camera):
    """src/bin/raysnail.rs:351-373: each SDL light -> Sphere(loc, 12, DiffuseLight(color) x1.7) in both lists."""
    lights = HittableList()
    for loc, col in lights_at:
        rs = Sphere(loc, 12.0, DiffuseLight(col).multiplier(1.7))
        lights.add(rs)
        hittables.add(rs)
    return World(hittables, lights, Gradient(C32(0.3, 0.4, 0.5), C32(0.7, 0.89, 1.0)), (0.0, camera.shutter_speed))


def _cli_camera(location, look_at, angle, width, height):
    """src/bin/raysnail.rs:340-349"""
    return CameraBuilder().look_from(location).look_at(look_at).fov(angle).aperture(0.01).focus(10.0) \
        .width(width).height(height).build()


def sdl_checker(c1: Color, c2: Color) -> Checker:
    """sdl_parser.rs pigment { checker c1, c2 } -> Checker::new(c1, c2, 2.0)"""
    return Checker(c1, c2, 2.0)


def example_sdl(width: int = 800, height: int = 500):
    """sdl/example.sdl:7-75 through the CLI (src/bin/raysnail.rs:311-386)."""
    cam = _cli_camera(Point3(6.0, 1.0, 2.5), Point3(0.0, -0.8, 0.0), 50.0, width, height)
    h = HittableList()
    h.add(Sphere((1.0, 0.0, -0.7), 1.0, Lambertian(C32(0.9, 0.5, 0.1))))
    h.add(Sphere((0.0, 1.0, 1.0), 0.7, Lambertian(C32(0.4, 0.8, 0.1))))
    h.add(Box((-2.0, -1.0, -4.0), (2.0, -0.75, -3.5), Lambertian(C32(0.1, 0.3, 0.7))))
    h.add(Box((1.5, -1.0, 2.5), (2.0, 0.0, 3.0), Lambertian(C32(0.1, 0.2, 0.6))))
    h.add(Box((-3.5, -1.2, -6.0), (3.5, -1.0, 4.0),
              Lambertian(sdl_checker(C32(0.3, 0.3, 0.3), C32(0.01, 0.01, 0.01)))))
    h.add(Sphere((0.0, -10002.0, 0.0), 10000.0, Lambertian(C32(0.07, 0.06, 0.05))))
    world = _cli_world(h, [((300.0, 400.0, 100.0), C32(1.0, 0.9, 0.7))], cam)
    return cam, world


def _translated(obj, t):
    st = TransformStack()
    st.push(Transform.translate(t))
    return TfFacade(obj, st)


def _quad(v1, v2, v3, j):
    """sdl_parser.rs:660: Quadric::new(v1.x, v2.x, v2.y, v3.x, v1.y, v2.z, v3.y, v1.z, v3.z, j)"""
    return Quadric(v1[0], v2[0], v2[1], v3[0], v1[1], v2[2], v3[1], v1[2], v3[2], j, None)


def quadric_sdl(width: int = 1024, height: int = 1024, cornell_emitter: bool = True):
    """sdl/quadric.sdl:8-107 through the CLI; with cornell_emitter the Cornell xz area light
    (examples/common/scene.rs:249-252, x15) is added to world and lights (config C4)."""
    cam = _cli_camera(Point3(10.0, 2.0, 4.0), Point3(0.0, -0.5, 1.0), 40.0, width, height)
    h = HittableList()
    specs = [
        (((1, 0, 1), (0, 0, 0), (0, -1, 0), 0.0), ((-1, -1, -1), (1, 1, 1)), C32(0.8, 0.7, 0.5), (1, -1, 4)),
        (((1.0, -1.0, 1.0), (0, 0, 0), (0, 0, 0), 0.0), ((-1, -1, -1), (1, 1, 1)), C32(0.7, 0.8, 0.5), (-1, 0, 2)),
        (((1.0, 0, 1.0), (0, 0, 0), (0, 0, 0), -1.0), ((-1, -1, -1), (1, 1, 1)), C32(0.5, 0.8, 0.7), (1, 0, 0)),
        (((1.0, -1.0, 1.0), (0, 0, 0), (0, 0, 0), -1.0), ((-2, -1, -2), (2, 1, 2)), C32(0.4, 0.6, 0.8), (-1, 0, -4)),
    ]
    for (v1, v2, v3, j), (b0, b1), col, tr in specs:
        q = _quad(tuple(map(float, v1)), tuple(map(float, v2)), tuple(map(float, v3)), float(j))
        bx = Box(tuple(map(float, b0)), tuple(map(float, b1)), None)
        inter = Intersection(q, bx, Lambertian(col))
        h.add(_translated(inter, tuple(map(float, tr))))
    h.add(Box((-3.5, -1.2, -8.0), (3.5, -1.0, 6.0),
              Lambertian(sdl_checker(C32(0.3, 0.3, 0.3), C32(0.01, 0.01, 0.01)))))
    h.add(Sphere((0.0, -10002.0, 0.0), 10000.0, Lambertian(C32(0.07, 0.06, 0.05))))
    world = _cli_world(h, [((50.0, 200.0, 200.0), C32(1.0, 0.9, 0.7))], cam)
    if cornell_emitter:
        rect = AARect.new_xz(AARectMetrics(554.0, (213.0, 343.0), (227.0, 332.0)),
                             DiffuseLight(C32(1.0, 1.0, 1.0)).multiplier(15.0))
        world.hittables.add(rect)
        world.lights.add(rect)
    return cam, world


def cornell_box(width: int = 600, height: int = 600, rotated: bool = True):
    """examples/common/scene.rs:211-334 (carton = true, smoke = false) with the emitter as the light."""
    red = Lambertian(C32(0.65, 0.05, 0.05))
    green = Lambertian(C32(0.12, 0.45, 0.15))
    white = Lambertian(C32(0.73, 0.73, 0.73))
    light = DiffuseLight(C32(1.0, 1.0, 1.0)).multiplier(15.0)
    o = HittableList()
    o.add(AARect.new_yz(AARectMetrics(555.0, (0.0, 555.0), (0.0, 555.0)), green))
    o.add(AARect.new_yz(AARectMetrics(0.0, (0.0, 555.0), (0.0, 555.0)), red))
    o.add(AARect.new_xz(AARectMetrics(0.0, (0.0, 555.0), (0.0, 555.0)), white))
    o.add(AARect.new_xz(AARectMetrics(555.0, (0.0, 555.0), (0.0, 555.0)), white))
    o.add(AARect.new_xy(AARectMetrics(555.0, (0.0, 555.0), (0.0, 555.0)), white))
    lrect = AARect.new_xz(AARectMetrics(554.0, (213.0, 343.0), (227.0, 332.0)), light)
    o.add(lrect)
    if rotated:
        s1 = TransformStack(); s1.push(Transform.rotate_by_y_axis(-18.0)); s1.push(Transform.translate((130.0, 0.0, 65.0)))
        s2 = TransformStack(); s2.push(Transform.rotate_by_y_axis(15.0)); s2.push(Transform.translate((265.0, 0.0, 295.0)))
        o.add(TfFacade(Box((0.0, 0.0, 0.0), (165.0, 165.0, 165.0), white), s1))
        o.add(TfFacade(Box((0.0, 0.0, 0.0), (165.0, 330.0, 165.0), white), s2))
    else:
        o.add(Box((130.0, 0.0, 65.0), (295.0, 165.0, 230.0), white))
        o.add(Box((265.0, 0.0, 295.0), (430.0, 330.0, 460.0), white))
    cam = CameraBuilder().fov(40.0).look_from(Point3(278.0, 278.0, -800.0)).look_at(Point3(278.0, 278.0, 0.0)) \
        .width(width).height(height).build()
    lights = HittableList()
    lights.add(lrect)
    return cam, World(o, lights, Gradient(C32(0.0, 0.0, 0.0), C32(0.0, 0.0, 0.0)), (0.0, 0.0))


def synthetic_mesh(n_theta: int = 120, n_phi: int = 300, seed: int = 1) -> Tuple[np.ndarray, np.ndarray]:
    """Deterministic bumpy closed mesh (~2*n_theta*n_phi triangles) standing in for the Stanford
    bunny (no OBJ file offline). Vertex normals follow triangle_mesh.rs:196-253 (area-unweighted
    sum of unit face normals, then unit)."""
    rng = np.random.default_rng(seed)
    th = np.linspace(0.0, np.pi, n_theta + 1)
    ph = np.linspace(0.0, 2.0 * np.pi, n_phi, endpoint=False)
    T, P = np.meshgrid(th, ph, indexing="ij")
    bumps = 1.0 + 0.08 * np.sin(5 * T) * np.cos(7 * P) + 0.02 * rng.standard_normal(T.shape)
    bumps[0, :] = bumps[0, 0]
    bumps[-1, :] = bumps[-1, 0]
    X = bumps * np.sin(T) * np.cos(P)
    Y = bumps * np.cos(T) * 0.9 + 1.0
    Z = bumps * np.sin(T) * np.sin(P)
    V = np.stack([X, Y, Z], -1).reshape(-1, 3)
    idx = lambda i, j: i * n_phi + (j % n_phi)
    tris = []
    for i in range(n_theta):
        for j in range(n_phi):
            a, b, c, d = idx(i, j), idx(i + 1, j), idx(i + 1, j + 1), idx(i, j + 1)
            if i != n_theta - 1:
                tris.append((a, b, c))
            if i != 0:
                tris.append((a, c, d))
    F = np.array(tris, dtype=np.int64)
    p0, p1, p2 = V[F[:, 0]], V[F[:, 1]], V[F[:, 2]]
    fn = np.cross(p1 - p0, p2 - p0)
    fn /= np.linalg.norm(fn, axis=1, keepdims=True)
    vn = np.zeros_like(V)
    for k in range(3):
        np.add.at(vn, F[:, k], fn)
    vn /= np.maximum(np.linalg.norm(vn, axis=1, keepdims=True), 1e-300)
    pos = np.concatenate([p0, p1, p2], axis=1)
    nrm = np.concatenate([vn[F[:, 0]], vn[F[:, 1]], vn[F[:, 2]]], axis=1)
    return pos, nrm


def mesh_scene(width: int = 1920, height: int = 1080, n_theta: int = 120, n_phi: int = 300):
    """Config C5: synthetic mesh + ground sphere + light sphere, camera as examples/preview_sdl2.rs:455-462."""
    pos, nrm = synthetic_mesh(n_theta, n_phi)
    h = HittableList()
    h.add(TriangleMesh(pos, nrm, Lambertian(C32(0.8, 0.6, 0.4))))
    h.add(Sphere((0.0, -1000.0, 0.0), 1000.0, Lambertian(C32(0.5, 0.5, 0.5))))
    lights = HittableList()
    light = Sphere((300.0, 400.0, 100.0), 12.0, DiffuseLight(C32(1.0, 0.9, 0.7)).multiplier(1.5))
    lights.add(light)
    h.add(light)
    cam = CameraBuilder().look_from(Point3(0.0, 2.0, 5.0)).look_at(Point3(0.0, 0.9, 0.0)).fov(40.0) \
        .width(width).height(height).build()
    return cam, World(h, lights, Gradient(C32(0.3, 0.4, 0.5), C32(0.7, 0.89, 1.0)), (0.0, 0.0))


def deep_spheres(width: int = 800, height: int = 500, n: int = 40000, seed: int = 5):
    """A synthetic spheres-only scene whose 4-wide tree is deep (not a reference scene: a stress case for the
    spheres mode's traversal stack past its LDS part): n small Lambertian / Metal spheres scattered over a
    60 x 60 field at random heights, the RTIOW ground, light and camera."""
    g = np.random.default_rng(seed)
    h = HittableList()
    h.add(Sphere((0.0, -1000.0, 0.0), 1000.0, Lambertian(C32(0.5, 0.5, 0.5))))
    xyz = g.uniform((-30.0, 0.0, -30.0), (30.0, 3.0, 30.0), size=(n, 3))
    rad = g.uniform(0.03, 0.15, size=n)
    kind = g.uniform(size=n)
    col = g.uniform(0.1, 0.9, size=(n, 3))
    for k in range(n):
        c = tuple(float(v) for v in xyz[k])
        if kind[k] < 0.85:
            mat = Lambertian(C32(*col[k]))
        else:
            mat = Metal(C32(*col[k]))
        h.add(Sphere(c, float(rad[k]), mat))
    lights = HittableList()
    light = Sphere((300.0, 400.0, 100.0), 12.0, DiffuseLight(C32(1.0, 0.9, 0.7)).multiplier(1.5))
    lights.add(light)
    h.add(light)
    cam = balls_scene_camera().width(width).height(height).build()
    return cam, World(h, lights, Gradient(C32(0.3, 0.4, 0.5), C32(0.7, 0.89, 1.0)), (0.0, cam.shutter_speed))


def cornell_smoke(width: int = 600, height: int = 600):
    """cornell_box_scene(carton = true, carton_rotation = true, smoke = true) (scene.rs:211-334): the
    light x7 over the larger rect, the two rotated boxes as ConstantMedium(white / black, 0.01)."""
    red = Lambertian(C32(0.65, 0.05, 0.05))
    green = Lambertian(C32(0.12, 0.45, 0.15))
    white = Lambertian(C32(0.73, 0.73, 0.73))
    light = DiffuseLight(C32(1.0, 1.0, 1.0)).multiplier(7.0)
    o = HittableList()
    o.add(AARect.new_yz(AARectMetrics(555.0, (0.0, 555.0), (0.0, 555.0)), green))
    o.add(AARect.new_yz(AARectMetrics(0.0, (0.0, 555.0), (0.0, 555.0)), red))
    o.add(AARect.new_xz(AARectMetrics(0.0, (0.0, 555.0), (0.0, 555.0)), white))
    o.add(AARect.new_xz(AARectMetrics(555.0, (0.0, 555.0), (0.0, 555.0)), white))
    o.add(AARect.new_xy(AARectMetrics(555.0, (0.0, 555.0), (0.0, 555.0)), white))
    lrect = AARect.new_xz(AARectMetrics(554.0, (113.0, 443.0), (127.0, 432.0)), light)
    o.add(lrect)
    s1 = TransformStack(); s1.push(Transform.rotate_by_y_axis(-18.0)); s1.push(Transform.translate((130.0, 0.0, 65.0)))
    s2 = TransformStack(); s2.push(Transform.rotate_by_y_axis(15.0)); s2.push(Transform.translate((265.0, 0.0, 295.0)))
    box1 = TfFacade(Box((0.0, 0.0, 0.0), (165.0, 165.0, 165.0), white), s1)
    box2 = TfFacade(Box((0.0, 0.0, 0.0), (165.0, 330.0, 165.0), white), s2)
    o.add(ConstantMedium(box1, C32(1.0, 1.0, 1.0), 0.01))
    o.add(ConstantMedium(box2, C32(0.0, 0.0, 0.0), 0.01))
    cam = CameraBuilder().fov(40.0).look_from(Point3(278.0, 278.0, -800.0)).look_at(Point3(278.0, 278.0, 0.0)) \
        .width(width).height(height).build()
    lights = HittableList()
    lights.add(lrect)
    return cam, World(o, lights, Gradient(C32(0.0, 0.0, 0.0), C32(0.0, 0.0, 0.0)), (0.0, 0.0))


def synthetic_image(width: int = 1920, height: int = 960, seed: int = 3) -> Image:
    """A deterministic RGB image standing in for examples/earth-map.png where the reference tree is
    absent (the GPU box): smooth bands plus noise, every byte value used."""
    rng = np.random.default_rng(seed)
    y, x = np.mgrid[0:height, 0:width]
    r = (127.5 + 127.5 * np.sin(x * 6.283185307179586 / width * 3.0)).astype(np.uint8)
    g = (y * 255 // max(1, height - 1)).astype(np.uint8)
    b = rng.integers(0, 256, (height, width), dtype=np.uint8)
    return Image(np.stack([r, g, b], -1))


EARTH_MAP = "/root/reference/examples/earth-map.png"


def all_feature_scene(width: int = 800, height: int = 800, seed: int = 7, perlin_seed: int = 1, earth: Image = None):
    """examples/common/scene.rs:336-469 (the book-2 final scene): 20x20 ground boxes in a BVH,
    the xz light x7, a moving sphere, glass, metal, a glass sphere filled with ConstantMedium, a
    global mist ConstantMedium, the earth-map sphere and a Perlin sphere. Upstream computes the
    rotated 1000-sphere group but never adds it (scene.rs:452-458), so it is not here either.
    Camera (478, 278, -600) -> (278, 278, 0), fov 40, shutter 1 (scene.rs:460-466); World time
    range 0..1; lights = the xz rect; black background."""
    rng = SeedRandom(seed)
    ground = Lambertian(C32(0.48, 0.83, 0.53))
    boxes1 = HittableList()
    for i in range(20):
        for j in range(20):
            w = 100.0
            x0, z0, y0 = -1000.0 + i * w, -1000.0 + j * w, 0.0
            y1 = rng.range(1.0, 100.0)
            boxes1.add(Box((x0, y0, z0), (x0 + w, y1, z0 + w), ground))
    o = HittableList()
    o.add(BVH(boxes1, (0.0, 1.0)))
    light = AARect.new_xz(AARectMetrics(554.0, (123.0, 423.0), (147.0, 412.0)),
                          DiffuseLight(C32(1.0, 1.0, 1.0)).multiplier(7.0))
    o.add(light)
    o.add(Sphere((400.0, 400.0, 200.0), 50.0, Lambertian(C32(0.7, 0.3, 0.1))).with_speed((30.0, 0.0, 0.0)))
    o.add(Sphere((260.0, 150.0, 45.0), 50.0, Dielectric(C32(1.0, 1.0, 1.0), 1.5).reflect_curve(Glass())))
    o.add(Sphere((0.0, 150.0, 145.0), 50.0, Metal(C32(0.8, 0.8, 0.9))))
    o.add(Sphere((360.0, 170.0, 145.0), 70.0, Dielectric(C32(1.0, 1.0, 1.0), 1.5).reflect_curve(Glass())))
    o.add(ConstantMedium(Sphere((360.0, 170.0, 145.0), 70.0, Lambertian(C32(1.0, 1.0, 1.0))),
                         C32(0.2, 0.4, 0.9), 0.2))
    o.add(ConstantMedium(Sphere((0.0, 0.0, 0.0), 5000.0, Dielectric(C32(1.0, 1.0, 1.0), 1.5).reflect_curve(Glass())),
                         C32(1.0, 1.0, 1.0), 0.0001))
    if earth is None:
        earth = Image.new(EARTH_MAP) if os.path.exists(EARTH_MAP) else synthetic_image()
    o.add(Sphere((400.0, 200.0, 400.0), 100.0, Lambertian(earth)))
    tex = Perlin(256, True, perlin_seed).scale(0.1).smooth(SmoothType.HermitianCubic)
    o.add(Sphere((220.0, 280.0, 300.0), 80.0, Lambertian(tex)))
    cam = CameraBuilder().look_from(Point3(478.0, 278.0, -600.0)).look_at(Point3(278.0, 278.0, 0.0)).fov(40.0) \
        .shutter_speed(1.0).width(width).height(height).build()
    lights = HittableList()
    lights.add(light)
    return cam, World(o, lights, Gradient(C32(0.0, 0.0, 0.0), C32(0.0, 0.0, 0.0)), (0.0, 1.0))


def materials_scene(width: int = 96, height: int = 64):
    """Build-owned parity fixture: BlinnPhong (material settings with phong), Perlin in all three
    types and smoothings (float and vector values), an Image texture on a sphere and on a rect,
    an Isotropic medium inside a glass sphere, a Difference, a checker ground and a light sphere."""
    h = HittableList()
    h.add(Sphere((0.0, -1000.0, 0.0), 1000.0, Lambertian(Checker(C32(0.2, 0.3, 0.1), C32(0.9, 0.9, 0.9), 10.0))))
    h.add(Sphere((-4.0, 1.0, 0.0), 1.0, BlinnPhong(0.5, 4.0, C32(0.99, 0.69, 0.2))))
    h.add(Sphere((-2.0, 0.6, 2.0), 0.6, BlinnPhong(0.2, 40.0, Perlin(64, False, 5).smooth(SmoothType.None_).scale(3.0))))
    h.add(Sphere((0.0, 1.0, 0.0), 1.0, Lambertian(Perlin(256, True, 2).scale(4.0).marble(5))))
    h.add(Sphere((2.0, 0.7, 2.2), 0.7, Lambertian(Perlin(128, True, 9).turbulence(7))))
    h.add(Sphere((0.5, 0.5, 2.8), 0.5, Lambertian(Perlin(32, False, 4).smooth(SmoothType.LinearInterpolate).scale(5.0))))
    img = synthetic_image(64, 32, seed=11)
    h.add(Sphere((4.0, 1.0, 0.0), 1.0, Lambertian(img)))
    h.add(AARect.new_xy(AARectMetrics(-3.0, (-6.0, 6.0), (0.0, 4.0)), Lambertian(img)))
    glass = Sphere((2.0, 1.2, -1.5), 1.2, Dielectric(C32(1.0, 1.0, 1.0), 1.5).reflect_curve(Glass()))
    h.add(glass)
    h.add(ConstantMedium(Sphere((2.0, 1.2, -1.5), 1.2, None), C32(0.2, 0.4, 0.9), 1.5))
    h.add(Difference(Box((-1.5, 0.0, -2.5), (-0.5, 1.0, -1.5), Lambertian(C32(0.8, 0.2, 0.2))),
                     Sphere((-1.0, 1.0, -2.0), 0.6, None), None))
    lights = HittableList()
    light = Sphere((10.0, 12.0, 8.0), 3.0, DiffuseLight(C32(1.0, 0.9, 0.7)).multiplier(4.0))
    lights.add(light)
    h.add(light)
    cam = CameraBuilder().look_from(Point3(9.0, 3.0, 7.0)).look_at(Point3(0.0, 0.8, 0.0)).fov(35.0) \
        .aperture(0.02).focus(10.0).width(width).height(height).build()
    return cam, World(h, lights, Gradient(C32(0.3, 0.4, 0.5), C32(0.7, 0.89, 1.0)), (0.0, 0.0))
