"""CPU: the BVH commit builds for any scene size (host-only commits, rs_scene_commit_devices(n = 0)).

The traversal stack keeps kStackMax entries in LDS and the rest in an HBM overflow array sized from
the tree's exact worst-case depth (rs_scene_info.stack_need), so neither deep SAH trees nor large
meshes are refused: C5's mesh and a ~1M-triangle mesh get the 4-wide tree, a skewed scene whose
SAH tree peels one object per level commits too.
"""
import numpy as np
import pytest

from raysnail_amd import _abi as A
from raysnail_amd import api, scenes
from raysnail_amd.scenes import C32
from raysnail_amd.api import (DiffuseLight, Gradient, HittableList, Lambertian, Sphere,
                              World)


def _info(world):
    return api.DeviceScene(world, devices=[]).info()


def test_c5_mesh_gets_the_4wide_tree():
    _, world = scenes.mesh_scene(64, 36)
    i = _info(world)
    assert i.n_objects == 71402 and i.n_world == 71402   # a mesh adds one leaf per triangle
    assert i.tree_arity == 4 and i.ref_order == 0 and i.scene_mode == 2   # flat mode
    assert i.stack_lds == 16 and 24 < i.stack_need < 64   # flat mode: 16 LDS entries (rs_internal.h stack_lds)
    assert i.n_devices == 0


def test_million_triangle_mesh_commits():
    _, world = scenes.mesh_scene(48, 27, 500, 1000)
    i = _info(world)
    assert i.n_objects == 998002 and i.tree_arity == 4 and i.stack_need < 128


def test_skewed_deep_scene_commits():
    """Spheres whose sizes double along a line: SAH splits off one object per level near the root."""
    h = HittableList()
    mat = Lambertian(C32(0.5, 0.5, 0.5))
    x = 0.0
    for k in range(40):
        r = 1.5 ** k * 1e-3
        h.add(Sphere((x + r, 0.0, 0.0), r, mat))
        x += 2.0 * r + 1e-6
    rng = np.random.default_rng(1)
    pts = rng.uniform(-1, 1, (20000, 3))
    for p in pts:
        h.add(Sphere(tuple(p), 1e-3, mat))
    lights = HittableList()
    lamp = Sphere((0.0, 50.0, 0.0), 1.0, DiffuseLight(C32(1.0, 1.0, 1.0)))
    lights.add(lamp)
    h.add(lamp)
    i = _info(World(h, lights, Gradient(C32(0.3, 0.4, 0.5), C32(0.7, 0.89, 1.0))))
    assert i.tree_arity == 4 and i.stack_need >= 1


def test_reference_order_scene_reports_inorder_4wide_tree():
    """Reference-order scenes (Box / Quadric / CSG) run on the in-order 4-wide collapse of the
    reference's tree (rs_host.cpp collapse4_inorder): one stack entry per entered inner child before
    slot 3, so the worst-case stack is at most the 4-wide depth."""
    _, world = scenes.quadric_sdl(32, 32)
    i = _info(world)
    assert i.tree_arity == 4 and i.ref_order == 1
    assert 1 <= i.stack_need <= i.tree_depth


def test_info_before_commit_is_a_state_error(hip_lib):
    import ctypes as C
    h = C.c_void_p()
    assert hip_lib.rs_scene_create(C.byref(h)) == 0
    inf = A.rs_scene_info()
    assert hip_lib.rs_scene_get_info(h, C.byref(inf)) == A.RS_E_STATE
    assert hip_lib.rs_scene_commit_devices(h, None, -1) == A.RS_E_INVALID
    assert hip_lib.rs_scene_destroy(h) == 0


def test_shading_classes_of_composites():
    """Host-only commit (no GPU): the material-sorted wavefront's class of a leaf object is its
    material's; composite objects (CSG, TfFacades of CSG) go to the generic class 4 even when every
    record they can produce is one class (quadric.sdl's translated quadric-box intersections), so
    the class queues keep CSG hits apart from leaf hits (rs_host.cpp RS_COMPOSITE_CLASS4); a CSG
    whose child brings its own light material is class 4 either way."""
    import sys, os
    sys.path.insert(0, os.path.dirname(__file__))
    from raysnail_amd.api import DeviceScene
    from raysnail_amd import scenes
    from test_gpu_parity import _emissive_csg_scene
    _, world = scenes.quadric_sdl(64, 64)
    info = DeviceScene(world, devices=[]).info()
    assert info.scene_mode == 4 and info.class_mask == 0b10001
    _, world = _emissive_csg_scene()
    info = DeviceScene(world, devices=[]).info()
    assert info.class_mask == 0b10001
