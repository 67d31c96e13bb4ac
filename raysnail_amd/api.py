"""Host-side mirror of raysnail's render-path API over the C-ABI.

Names, argument meaning and error behaviour follow the reference so that code written against
raysnail reads the same:

    camera = CameraBuilder().look_from(Point3(13, 2, 3)).look_at(Point3(0, 0, 0)).fov(20.0) \\
        .aperture(0.02).focus(10.0).width(800).height(500).build()        # src/camera.rs:300-413
    world = World(hittables, lights, background=Gradient(...), time_range=(0.0, camera.shutter_speed))
    pixels = camera.take_photo().samples(122).depth(8).shot(None, world)   # src/camera.rs:113-295

Geometry / materials are plain descriptions (the reference's Arc<dyn ...> objects); they are
realised into a device scene the first time a World is rendered. The realisation is generic over
a backend `lib` + symbol prefix so tests can replay the identical scene into the CPU oracle.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass, field
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np

from . import _abi as A


class RaysnailError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


# ----------------------------------------------------------------------------- prelude ----
def Point3(x: float, y: float, z: float) -> Tuple[float, float, float]:
    return (float(x), float(y), float(z))


Vec3 = Point3


@dataclass(frozen=True)
class Color:
    """src/prelude/color.rs:11-16 (f32 rgba)."""
    r: float
    g: float
    b: float
    a: float = 1.0


# ----------------------------------------------------------------------------- textures ----
@dataclass(eq=False)
class Checker:
    """src/texture/checker.rs:13-30: sin(s x) sin(s y) sin(s z) < 0 -> odd else even."""
    odd: Color
    even: Color
    scale: float


class SmoothType:                    # src/texture/noise.rs:4-9
    None_ = A.RS_SMOOTH_NONE
    LinearInterpolate = A.RS_SMOOTH_LINEAR
    HermitianCubic = A.RS_SMOOTH_HERMITE


class Perlin:
    """src/texture/noise.rs. Perlin::new(point_count, vector, rng) draws its tables from a FastRng the
    reference seeds from the OS; here the FastRng seed is explicit (tables built by the C++ host
    layer: Vec3::random_unit / gen values, rand 0.8 shuffles)."""

    def __init__(self, point_count: int, vector: bool, rng_seed: int):
        from . import host_lib
        self.point_count, self.vector = int(point_count), bool(vector)
        self.values, self.perms = host_lib.perlin_tables(int(rng_seed), self.point_count, self.vector)
        self._scale, self._smooth, self._type, self._depth = 1.0, SmoothType.HermitianCubic, A.RS_PERLIN_NORMAL, 0

    def scale(self, s):
        self._scale = float(s); return self

    def smooth(self, t):
        self._smooth = int(t); return self

    def turbulence(self, depth: int):
        self._type, self._depth = A.RS_PERLIN_TURBULENCE, int(depth); return self

    def marble(self, depth: int):
        self._type, self._depth = A.RS_PERLIN_MARBLE, int(depth); return self


class Image:
    """src/texture/image.rs: decoded 8-bit RGB pixels, row 0 = top."""

    def __init__(self, rgb: np.ndarray):
        rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
        assert rgb.ndim == 3 and rgb.shape[2] == 3, "H x W x 3 uint8 expected"
        self.rgb = rgb

    @staticmethod
    def new(path: str) -> "Image":
        """Image::new (image.rs:24-31): PNG decode by the C++ host layer."""
        from . import host_lib
        return Image(host_lib.png_load(path))


def _tex_desc(t, data: int = 0) -> A.rs_texture_desc:
    d = A.rs_texture_desc()
    d.data = data
    if isinstance(t, (Perlin, Image)):
        d.kind = A.RS_TEX_PERLIN if isinstance(t, Perlin) else A.RS_TEX_IMAGE
        d.even[:] = [1.0, 1.0, 1.0, 1.0]
        d.odd[:] = [1.0, 1.0, 1.0, 1.0]
        d.scale = 1.0
    elif isinstance(t, Color):
        d.kind = A.RS_TEX_SOLID
        d.even[:] = [t.r, t.g, t.b, t.a]
        d.odd[:] = [t.r, t.g, t.b, t.a]
        d.scale = 1.0
    elif isinstance(t, Checker):
        d.kind = A.RS_TEX_CHECKER
        d.even[:] = [t.even.r, t.even.g, t.even.b, t.even.a]
        d.odd[:] = [t.odd.r, t.odd.g, t.odd.b, t.odd.a]
        d.scale = float(t.scale)
    else:
        raise TypeError(f"unsupported texture {type(t).__name__}")
    return d


# ----------------------------------------------------------------------------- materials ----
@dataclass
class CommonMaterialSettings:
    """src/material/mod.rs:41-54"""
    phong_factor: float = 0.0
    phong_exponent: int = 1


class Material:
    settings: CommonMaterialSettings

    def set(self, settings: CommonMaterialSettings):
        self.settings = settings
        return self


class Lambertian(Material):          # src/material/lambertian.rs
    def __init__(self, texture):
        self.texture, self.settings = texture, CommonMaterialSettings()


class Metal(Material):               # src/material/metal.rs:86-118
    def __init__(self, texture):
        self.texture, self.settings = texture, CommonMaterialSettings()


class DiffuseMetal(Material):        # src/material/metal.rs:36-68
    def __init__(self, exponent: float, texture):
        self.exponent, self.texture, self.settings = float(exponent), texture, CommonMaterialSettings()


class Glass:                         # src/material/dielectric.rs:17-25 (Schlick curve)
    pass


class Dielectric(Material):          # src/material/dielectric.rs:27-93
    def __init__(self, color: Color, refractive: float):
        self.color, self.refractive, self.glass = color, float(refractive), False
        self.settings = CommonMaterialSettings()

    def reflect_curve(self, curve):
        if not isinstance(curve, Glass):
            raise TypeError("only the Glass reflect curve exists upstream")
        self.glass = True
        return self


class DiffuseLight(Material):        # src/material/light.rs
    def __init__(self, texture):
        self.texture, self.mult, self.settings = texture, 1.0, CommonMaterialSettings()

    def multiplier(self, m: float):
        self.mult = float(m)
        return self


class Isotropic(Material):           # src/material/isotropic.rs
    def __init__(self, color: Color):
        self.color, self.settings = color, CommonMaterialSettings()


class BlinnPhong(Material):          # src/material/blinn_phong.rs
    def __init__(self, k_specular: float, exponent: float, texture):
        self.k_specular, self.exponent, self.texture = float(k_specular), float(exponent), texture
        self.settings = CommonMaterialSettings()


class MixedMaterial(Material):       # src/material/mixed_material.rs
    def __init__(self, material_1: Material, material_2: Material, probability_1: float):
        self.m1, self.m2, self.p = material_1, material_2, float(probability_1)

    @property
    def settings(self):
        return self.m1.settings


# ----------------------------------------------------------------------------- geometry ----
class Hittable:
    pass


class Sphere(Hittable):              # src/hittable/geometry/sphere.rs
    def __init__(self, center, radius: float, material: Optional[Material]):
        self.center, self.radius, self.material = tuple(map(float, center)), float(radius), material
        self.speed = (0.0, 0.0, 0.0)

    def with_speed(self, speed):
        self.speed = tuple(map(float, speed))
        return self


@dataclass
class AARectMetrics:                 # src/hittable/geometry/rect.rs:17-37
    k: float
    a: Tuple[float, float]
    b: Tuple[float, float]

    def __post_init__(self):
        if not (self.a[0] < self.a[1] and self.b[0] < self.b[1]):
            raise ValueError("AARectMetrics requires a0 < a1 and b0 < b1 (rect.rs:27-28)")


class AARect(Hittable):              # src/hittable/geometry/rect.rs
    def __init__(self, plane: int, metrics: AARectMetrics, material: Optional[Material]):
        self.plane, self.metrics, self.material = plane, metrics, material

    @classmethod
    def new_xy(cls, m, mat):
        return cls(A.RS_PLANE_XY, m, mat)

    @classmethod
    def new_xz(cls, m, mat):
        return cls(A.RS_PLANE_XZ, m, mat)

    @classmethod
    def new_yz(cls, m, mat):
        return cls(A.RS_PLANE_YZ, m, mat)


class Box(Hittable):                 # src/hittable/geometry/box.rs
    def __init__(self, p0, p1, material: Optional[Material]):
        self.p0, self.p1, self.material = tuple(map(float, p0)), tuple(map(float, p1)), material


class Quadric(Hittable):             # src/hittable/geometry/quadric.rs (field order qa..qj)
    def __init__(self, qa, qb, qc, qd, qe, qf, qg, qh, qi, qj, material: Optional[Material]):
        self.q = tuple(map(float, (qa, qb, qc, qd, qe, qf, qg, qh, qi, qj)))
        self.material = material


class TriangleMesh(Hittable):        # src/hittable/geometry/triangle_mesh.rs (Triangle list)
    def __init__(self, positions: np.ndarray, normals: Optional[np.ndarray], material: Optional[Material]):
        self.positions = np.ascontiguousarray(positions, dtype=np.float64).reshape(-1, 9)
        self.normals = None if normals is None else np.ascontiguousarray(normals, dtype=np.float64).reshape(-1, 9)
        self.material = material

    @staticmethod
    def load(filename: str, scale: float, offset, rotation_angle: float, axis: int,
             material: Optional[Material]) -> "TriangleMesh":
        """TriangleMesh::load (triangle_mesh.rs:166-276): OBJ through the C++ host layer's
        tobj-compatible reader (single_index, triangulate)."""
        from . import host_lib
        pos, nrm = host_lib.obj_load(filename, scale, offset, rotation_angle, axis)
        return TriangleMesh(pos, nrm, material)


class ConstantMedium(Hittable):      # src/hittable/medium/constant.rs (material Isotropic(color))
    def __init__(self, boundary: Hittable, color: Color, density: float):
        self.boundary, self.color, self.density = boundary, color, float(density)


class BVH(Hittable):
    """A BVH / HittableList used as one object (bvh.rs, list.rs): the device scene has one BVH over
    every object, so the group exports its members (a TfFacade of a group transforms each member)."""

    def __init__(self, objects, time_limit=(0.0, 0.0)):
        self.objects = list(objects.objects if isinstance(objects, HittableList) else objects)


class Intersection(Hittable):        # src/hittable/csg/intersection.rs
    def __init__(self, o1: Hittable, o2: Hittable, material: Optional[Material]):
        self.o1, self.o2, self.material = o1, o2, material


class Difference(Hittable):          # src/hittable/csg/difference.rs
    def __init__(self, plus: Hittable, minus: Hittable, material: Optional[Material]):
        self.plus, self.minus, self.material = plus, minus, material


class Transform:                     # src/hittable/transform/transform.rs:16-107
    def __init__(self, kind: int, v):
        self.kind, self.v = kind, tuple(map(float, v))

    @staticmethod
    def translate(t):
        return Transform(A.RS_TF_TRANSLATE, t)

    @staticmethod
    def rotate_by_x_axis(theta):
        return Transform(A.RS_TF_ROTATE_X, (theta, 0, 0))

    @staticmethod
    def rotate_by_y_axis(theta):
        return Transform(A.RS_TF_ROTATE_Y, (theta, 0, 0))

    @staticmethod
    def rotate_by_z_axis(theta):
        return Transform(A.RS_TF_ROTATE_Z, (theta, 0, 0))

    @staticmethod
    def scale(t):
        return Transform(A.RS_TF_SCALE, t)


class TransformStack:                # src/hittable/transform/transform.rs:110-157
    def __init__(self):
        self.stack: List[Transform] = []

    def push(self, t: Transform):
        self.stack.append(t)

    def __len__(self):
        return len(self.stack)


class TfFacade(Hittable):            # src/hittable/transform/tf_facade.rs
    def __init__(self, obj: Hittable, stack: TransformStack):
        self.obj, self.stack = obj, stack


class HittableList:                  # src/hittable/collection/list.rs
    def __init__(self):
        self.objects: List[Hittable] = []

    def add(self, obj: Hittable):
        self.objects.append(obj)
        return self

    def __len__(self):
        return len(self.objects)


@dataclass
class Gradient:
    """The background closure used by every reference front-end: lo.gradient(hi, (d.y+1)*0.5)
    (examples/rtow_13_1.rs:38-41, src/bin/raysnail.rs:364-367, src/prelude/color.rs:50-58)."""
    lo: Color = Color(0.3, 0.4, 0.5)
    hi: Color = Color(0.7, 0.89, 1.0)


class World:                         # src/hittable/collection/world.rs
    def __init__(self, hittables: HittableList, lights: HittableList, background: Gradient = None,
                 time_range: Tuple[float, float] = (0.0, 0.0)):
        self.hittables, self.lights = hittables, lights
        self.background = background or Gradient()
        self.time_range = (float(time_range[0]), float(time_range[1]))
        self._scene = None

    def device_scene(self) -> "DeviceScene":
        if self._scene is None:
            self._scene = DeviceScene(self)
        return self._scene


# ----------------------------------------------------------------------------- realisation ----
def _check(lib, code: int, prefix: str):
    if code != 0:
        err = getattr(lib, prefix + "last_error")()
        raise RaysnailError(code, err.decode() if isinstance(err, bytes) else str(err))


def realize(world: World, lib, handle, prefix: str = "rs_") -> None:
    """Replay the world description into a backend scene (libraysnail_hip or the test oracle)."""
    mat_ids = {}
    obj_ids = {}
    tex_ids = {}

    def call(name, *args):
        _check(lib, getattr(lib, prefix + name)(handle, *args), prefix)

    def tex(t) -> A.rs_texture_desc:
        if not isinstance(t, (Perlin, Image)):
            return _tex_desc(t)
        if id(t) not in tex_ids:
            out = C.c_int32()
            if isinstance(t, Perlin):
                pd = A.rs_perlin_desc()
                pd.point_count, pd.vector, pd.smooth, pd.type = t.point_count, int(t.vector), t._smooth, t._type
                pd.depth, pd.scale = t._depth, t._scale
                pd.values = t.values.ctypes.data_as(C.POINTER(C.c_double))
                n = t.point_count
                pd.perm_x = t.perms[:n].ctypes.data_as(C.POINTER(C.c_uint32))
                pd.perm_y = t.perms[n:2 * n].ctypes.data_as(C.POINTER(C.c_uint32))
                pd.perm_z = t.perms[2 * n:].ctypes.data_as(C.POINTER(C.c_uint32))
                call("perlin", C.byref(pd), C.byref(out))
            else:
                h, w = t.rgb.shape[:2]
                call("image", t.rgb.ctypes.data_as(C.c_void_p), w, h, C.byref(out))
            tex_ids[id(t)] = out.value
        return _tex_desc(t, tex_ids[id(t)])

    def mat_id(m: Optional[Material]) -> int:
        if m is None:
            return A.RS_NO_MATERIAL
        if id(m) in mat_ids:
            return mat_ids[id(m)]
        d = A.rs_material_desc()
        d.refractive, d.exponent, d.multiplier, d.mix_p = 1.0, 0.0, 1.0, 0.5
        if isinstance(m, MixedMaterial):
            a, b = mat_id(m.m1), mat_id(m.m2)
            d.kind, d.mix_a, d.mix_b, d.mix_p = A.RS_MAT_MIXED, a, b, m.p
            d.texture = _tex_desc(Color(0, 0, 0))
        else:
            if isinstance(m, Lambertian):
                d.kind, d.texture = A.RS_MAT_LAMBERTIAN, tex(m.texture)
            elif isinstance(m, Metal):
                d.kind, d.texture = A.RS_MAT_METAL, tex(m.texture)
            elif isinstance(m, DiffuseMetal):
                d.kind, d.texture, d.exponent = A.RS_MAT_DIFFUSE_METAL, tex(m.texture), m.exponent
            elif isinstance(m, Dielectric):
                d.kind, d.texture, d.refractive, d.glass = A.RS_MAT_DIELECTRIC, _tex_desc(m.color), m.refractive, int(m.glass)
            elif isinstance(m, DiffuseLight):
                d.kind, d.texture, d.multiplier = A.RS_MAT_DIFFUSE_LIGHT, tex(m.texture), m.mult
            elif isinstance(m, Isotropic):
                d.kind, d.texture = A.RS_MAT_ISOTROPIC, _tex_desc(m.color)
            elif isinstance(m, BlinnPhong):
                d.kind, d.texture = A.RS_MAT_BLINN_PHONG, tex(m.texture)
                d.k_specular, d.exponent = m.k_specular, m.exponent
            else:
                raise TypeError(f"unsupported material {type(m).__name__}")
            d.phong_factor, d.phong_exponent = m.settings.phong_factor, int(m.settings.phong_exponent)
        out = C.c_int32()
        call("material", C.byref(d), C.byref(out))
        mat_ids[id(m)] = out.value
        return out.value

    def single(h):
        if isinstance(h, list):
            if len(h) != 1:
                raise RaysnailError(A.RS_E_UNSUPPORTED, "operand must be a single object")
            return h[0]
        return h

    def obj_id(o: Hittable) -> int:
        if id(o) in obj_ids:
            return obj_ids[id(o)]
        out = C.c_uint32()
        if isinstance(o, Sphere):
            call("sphere", A.D3(*o.center), o.radius, A.D3(*o.speed), mat_id(o.material), C.byref(out))
        elif isinstance(o, AARect):
            m = o.metrics
            call("aarect", o.plane, m.k, m.a[0], m.a[1], m.b[0], m.b[1], mat_id(o.material), C.byref(out))
        elif isinstance(o, Box):
            call("box", A.D3(*o.p0), A.D3(*o.p1), mat_id(o.material), C.byref(out))
        elif isinstance(o, Quadric):
            call("quadric", (C.c_double * 10)(*o.q), mat_id(o.material), C.byref(out))
        elif isinstance(o, TriangleMesh):
            pos = o.positions
            nrm = o.normals
            call("triangles", pos.ctypes.data_as(C.POINTER(C.c_double)),
                 None if nrm is None else nrm.ctypes.data_as(C.POINTER(C.c_double)),
                 pos.shape[0], mat_id(o.material), C.byref(out))
            obj_ids[id(o)] = list(range(out.value, out.value + pos.shape[0]))
            return obj_ids[id(o)]
        elif isinstance(o, Intersection):
            a, b = single(obj_id(o.o1)), single(obj_id(o.o2))
            call("intersection", a, b, mat_id(o.material), C.byref(out))
        elif isinstance(o, Difference):
            a, b = single(obj_id(o.plus)), single(obj_id(o.minus))
            call("difference", a, b, mat_id(o.material), C.byref(out))
        elif isinstance(o, ConstantMedium):
            b = single(obj_id(o.boundary))
            c = o.color
            call("constant_medium", b, (C.c_float * 4)(c.r, c.g, c.b, c.a), o.density, C.byref(out))
        elif isinstance(o, BVH):
            hs = []
            for m in o.objects:
                h = obj_id(m)
                hs.extend(h if isinstance(h, list) else [h])
            obj_ids[id(o)] = hs
            return hs
        elif isinstance(o, TfFacade):
            child = obj_id(o.obj)
            arr = (A.rs_transform * max(1, len(o.stack)))()
            for i, t in enumerate(o.stack.stack):
                arr[i].kind = t.kind
                arr[i].v[:] = list(t.v)
            if isinstance(child, list):  # a transformed mesh / group: each member transformed
                hs = []
                for c in child:
                    call("transformed", c, arr, len(o.stack), C.byref(out))
                    hs.append(out.value)
                obj_ids[id(o)] = hs
                return hs
            call("transformed", child, arr, len(o.stack), C.byref(out))
        else:
            raise TypeError(f"unsupported hittable {type(o).__name__}")
        obj_ids[id(o)] = out.value
        return out.value

    def add_list(lst: HittableList, fn: str):
        for o in lst.objects:
            h = obj_id(o)
            for hh in (h if isinstance(h, list) else [h]):
                call(fn, hh)

    bg = world.background
    call("set_background", A.F3(bg.lo.r, bg.lo.g, bg.lo.b), A.F3(bg.hi.r, bg.hi.g, bg.hi.b))
    call("set_time_range", world.time_range[0], world.time_range[1])
    add_list(world.hittables, "world_add")
    add_list(world.lights, "lights_add")


class DeviceScene:
    """A committed libraysnail_hip scene (BVH + SoA scene data resident in HBM)."""

    def __init__(self, world: World, devices: Optional[Sequence[int]] = None):
        """devices: None = the current HIP device (rs_scene_commit); a list of HIP ordinals (repeats
        allowed: virtual devices) = rs_scene_commit_devices; [] = host-only build (info() only)."""
        self.lib = A.load()
        h = C.c_void_p()
        _check(self.lib, self.lib.rs_scene_create(C.byref(h)), "rs_")
        self.handle = h
        realize(world, self.lib, h, "rs_")
        if devices is None:
            _check(self.lib, self.lib.rs_scene_commit(h), "rs_")
        else:
            devs = (C.c_int * max(1, len(devices)))(*devices)
            _check(self.lib, self.lib.rs_scene_commit_devices(h, devs, len(devices)), "rs_")

    def __del__(self):
        try:
            if self.handle:
                self.lib.rs_scene_destroy(self.handle)
                self.handle = None
        except Exception:
            pass

    def info(self) -> A.rs_scene_info:
        """What commit built: tree arity / depth, exact stack need, scene mode (rs_scene_get_info)."""
        inf = A.rs_scene_info()
        _check(self.lib, self.lib.rs_scene_get_info(self.handle, C.byref(inf)), "rs_")
        return inf

    def set_lanes(self, lanes: int) -> None:
        """Chunk lanes of the bounce-synchronous wavefront for later renders (rs_scene_set_lanes)."""
        _check(self.lib, self.lib.rs_scene_set_lanes(self.handle, lanes), "rs_")

    def set_frames_in_flight(self, frames: int) -> None:
        """Frame slots per device: asynchronous frames overlap (rs_scene_set_frames_in_flight)."""
        _check(self.lib, self.lib.rs_scene_set_frames_in_flight(self.handle, frames), "rs_")

    def set_workspace(self, max_batch_items: int = 0, pool_paths: int = 0) -> None:
        """Radiance batch size and path-set capacity, 0 = keep (rs_scene_set_workspace); scheduling only."""
        _check(self.lib, self.lib.rs_scene_set_workspace(self.handle, max_batch_items, pool_paths), "rs_")

    def render(self, cam: A.rs_camera_desc, st: A.rs_render_settings, mask: Optional[np.ndarray] = None,
               out: Optional[np.ndarray] = None) -> Tuple[np.ndarray, A.rs_render_stats]:
        H, W = cam.height, cam.width
        if out is None:
            out = np.zeros((H, W, 4), dtype=np.float32)
        assert out.shape == (H, W, 4) and out.dtype == np.float32 and out.flags.c_contiguous
        mptr = None
        if mask is not None:
            mask = np.ascontiguousarray(mask, dtype=np.uint8).reshape(H * W)
            mptr = mask.ctypes.data_as(C.c_void_p)
        stats = A.rs_render_stats()
        _check(self.lib, self.lib.rs_render(self.handle, C.byref(cam), C.byref(st), mptr,
                                            out.ctypes.data_as(C.c_void_p), C.byref(stats)), "rs_")
        return out, stats

    def render_rows(self, cam: A.rs_camera_desc, st: A.rs_render_settings, on_row, mask: Optional[np.ndarray] = None,
                    bands: int = 16, stats: bool = True) -> Tuple[np.ndarray, Optional[A.rs_render_stats]]:
        """rs_render_rows: on_row(y, out) is called for each lattice row y as soon as its band is complete
        (out[y] holds it), in lattice order, from this thread; then on_row(H, out) (the sentinel)."""
        H, W = cam.height, cam.width
        out = np.zeros((H, W, 4), dtype=np.float32)
        mptr = None
        if mask is not None:
            mask = np.ascontiguousarray(mask, dtype=np.uint8).reshape(H * W)
            mptr = mask.ctypes.data_as(C.c_void_p)
        err = []

        def cb(user, y, row, width):
            if err:
                return
            try:  # no exception may cross the C ABI: kept and raised after the call
                on_row(int(y), out)
            except BaseException as e:  # noqa: BLE001
                err.append(e)
        ccb = A.ROW_CALLBACK(cb)
        st_out = A.rs_render_stats() if stats else None
        _check(self.lib, self.lib.rs_render_rows(self.handle, C.byref(cam), C.byref(st), mptr,
                                                 out.ctypes.data_as(C.c_void_p), bands, ccb, None,
                                                 C.byref(st_out) if stats else None), "rs_")
        if err:
            raise err[0]
        return out, st_out

    def render_device(self, cam: A.rs_camera_desc, st: A.rs_render_settings, d_out_ptr: int,
                      stream_ptr: int = 0, d_mask_ptr: int = 0, stats: bool = True):
        """rs_render_device. stats=True: synchronous, returns rs_render_stats (kernel timing included);
        stats=False: returns None as soon as the frame is enqueued on the stream (asynchronous)."""
        out = A.rs_render_stats() if stats else None
        _check(self.lib, self.lib.rs_render_device(self.handle, C.byref(cam), C.byref(st), d_mask_ptr or None,
                                                   C.c_void_p(d_out_ptr), stream_ptr or None,
                                                   C.byref(out) if stats else None), "rs_")
        return out

    def render_device_passes(self, cam: A.rs_camera_desc, st: A.rs_render_settings, d_out_ptrs, stream_ptr: int = 0,
                             stats: bool = True):
        """rs_render_device_passes: passes st.pass + k into the device frames d_out_ptrs[k] (one sample stream on
        streaming scenes). stats as render_device."""
        n = len(d_out_ptrs)
        ptrs = (C.c_void_p * max(1, n))(*[C.c_void_p(p) for p in d_out_ptrs])
        out = A.rs_render_stats() if stats else None
        _check(self.lib, self.lib.rs_render_device_passes(self.handle, C.byref(cam), C.byref(st), n, ptrs,
                                                          stream_ptr or None, C.byref(out) if stats else None), "rs_")
        return out


# ----------------------------------------------------------------------------- camera ----
class Camera:
    """src/camera.rs:18-91 (the basis itself is computed inside the library, camera.rs:37-73)."""

    def __init__(self, desc: A.rs_camera_desc):
        self.desc = desc

    @property
    def shutter_speed(self) -> float:
        return self.desc.shutter

    @property
    def picture_width(self) -> int:
        return self.desc.width

    @property
    def picture_height(self) -> int:
        return self.desc.height

    def take_photo(self) -> "TakePhotoSettings":
        return TakePhotoSettings(self)


class CameraBuilder:
    """src/camera.rs:300-413 (defaults :314-329)."""

    def __init__(self):
        self._from, self._at, self._vup = (0.0, 0.0, 0.0), (0.0, 0.0, -1.0), (0.0, 1.0, 0.0)
        self._fov, self._aperture, self._focus, self._shutter = 90.0, 0.0, 1.0, 0.0
        self._w, self._h = 400, 200

    def look_from(self, p):
        self._from = tuple(map(float, p)); return self

    def look_at(self, p):
        self._at = tuple(map(float, p)); return self

    def vup(self, v):
        self._vup = tuple(map(float, v)); return self

    def fov(self, f):
        self._fov = float(f); return self

    def aperture(self, a):
        self._aperture = float(a); return self

    def focus(self, d):
        self._focus = float(d); return self

    def focus_to_look_at(self):
        d = [a - b for a, b in zip(self._at, self._from)]
        return self.focus(math.sqrt(math.fsum(x * x for x in d)))

    def shutter_speed(self, s):
        self._shutter = float(s); return self

    def width(self, w):
        self._w = int(w); return self

    def height(self, h):
        self._h = int(h); return self

    def build(self) -> Camera:
        d = A.rs_camera_desc()
        d.look_from[:] = list(self._from)
        d.look_at[:] = list(self._at)
        d.vup[:] = list(self._vup)
        d.fov, d.aperture, d.focus, d.shutter = self._fov, self._aperture, self._focus, self._shutter
        d.width, d.height = self._w, self._h
        return Camera(d)


class PainterTarget:                 # src/painter.rs:23-27
    def register_pixels(self, y: int, pixels) -> None:
        pass


class PainterController:             # src/painter.rs:28-32 (never polled upstream)
    def receive_command(self):
        return None


class PixelController:               # src/painter.rs:34-38
    def calculate_pixel(self, x: int, y: int) -> bool:
        return True


class TakePhotoSettings:
    """src/camera.rs:103-154 + the GPU-side painter knobs (seed/pass/rows/mode)."""

    def __init__(self, camera: Camera):
        self.camera = camera
        self._depth, self._gamma, self._samples = 8, True, 50
        self._seed, self._pass, self._mode = 0, 0, A.RS_MODE_AUTO
        self._rows = (0, 0, 1)

    def depth(self, d):
        self._depth = int(d); return self

    def gamma(self, g):
        self._gamma = bool(g); return self

    def samples(self, s):
        self._samples = int(s); return self

    def threads(self, _t):
        return self  # CPU-painter knob; meaningless on the GPU path

    def parallel(self, _p):
        return self

    def seed(self, s):
        self._seed = int(s); return self

    def pass_index(self, p):
        self._pass = int(p); return self

    def rows(self, begin: int, end: int = 0, step: int = 1):
        self._rows = (int(begin), int(end), int(step)); return self

    def mode(self, m: int):
        self._mode = int(m); return self

    def settings(self) -> A.rs_render_settings:
        st = A.rs_render_settings()
        st.samples, st.depth, st.gamma, st.mode = self._samples, self._depth, int(self._gamma), self._mode
        st.seed, st.pass_ = self._seed, self._pass
        st.row_begin, st.row_end, st.row_step = self._rows
        return st

    def shot_to_target(self, path, world: World, target: PainterTarget, controller: PainterController,
                       pixel_map: PixelController) -> np.ndarray:
        """src/camera.rs:261-287: returns the (H, W, 4) float32 frame, rows registered with target."""
        cam = self.camera.desc
        mask = None
        if pixel_map is not None and type(pixel_map) is not PixelController:
            mask = np.array([[1 if pixel_map.calculate_pixel(x, y) else 0 for x in range(cam.width)]
                             for y in range(cam.height)], dtype=np.uint8)
        st = self.settings()
        if target is None:
            out, stats = world.device_scene().render(cam, st, mask)
            self.last_stats = stats
            return out
        # progressive delivery (painter.rs:214 registers each row as a worker finishes it):
        # rs_render_rows hands each band of the row lattice over as soon as it is complete, later bands
        # still in flight; pixels do not depend on the banding (per-sample RNG streams), so the frame
        # equals the one-call frame. Rows off the lattice (all zero) are registered before the sentinel.
        H = cam.height
        sent = np.zeros(H, dtype=bool)

        def on_row(y, out):
            if y == H:
                for r in np.flatnonzero(~sent):
                    target.register_pixels(int(r), out[r])
                target.register_pixels(H, [])  # end-of-pass sentinel (painter.rs:332)
                return
            sent[y] = True
            target.register_pixels(y, out[y])
        out, self.last_stats = world.device_scene().render_rows(cam, st, on_row, mask)
        return out

    def shot(self, path, world: World) -> np.ndarray:
        """src/camera.rs:290-295 (path is ignored upstream too)."""
        return self.shot_to_target(path, world, None, None, None)
