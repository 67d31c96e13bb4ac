"""raysnail_amd — MI355X-native (gfx950) render path of raysnail (Varkalandar/raysnail).

The hot path (Painter sample loop -> Camera::ray -> Hittable::hit BVH -> Material::scatter /
emitted) runs as hand-written HIP kernels in libraysnail_hip.so behind the C-ABI declared in
include/raysnail_hip.h. This package is the host-side mirror of the reference's API over that
ABI (api.py) plus the scene builders for the benchmark configurations (scenes.py).
"""
from . import _abi  # noqa: F401
from .api import (AARect, AARectMetrics, Box, Camera, CameraBuilder, Checker, Color, CommonMaterialSettings,  # noqa: F401
                  Dielectric, Difference, DiffuseLight, DiffuseMetal, Glass, Gradient, HittableList, Intersection,
                  Lambertian, MixedMaterial, Metal, PainterController, PainterTarget, PixelController, Point3,
                  Quadric, RaysnailError, Sphere, TakePhotoSettings, TfFacade, Transform, TransformStack,
                  TriangleMesh, Vec3, World, realize)

__all__ = [n for n in dir() if not n.startswith("_")]
