"""libm semantics of the render path (include/rs_crmath.h): correctly rounded sin / cos / pow,
shared by the GPU kernels and the oracle.

* the implementation against libquadmath's 113-bit functions (an independent reference), on the
  argument ranges the path produces and on generic ones;
* what the choice changes: the oracle built on glibc 2.35's libm (liboracle_glibc.so, i.e. what
  raysnail itself computes on this image) against the correctly rounded oracle -- frames agree
  within the north-star tolerance (RMSE < 1e-4).
"""
import os
import subprocess

import numpy as np
import pytest

from raysnail_amd import scenes

HERE = os.path.dirname(os.path.abspath(__file__))


def test_crmath_against_quad_precision(tmp_path):
    exe = tmp_path / "test_crmath"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-o", str(exe),
                    os.path.join(HERE, "cpp", "test_crmath.cpp"), "-lquadmath"], check=True)
    r = subprocess.run([str(exe), "300000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.parametrize("name,build", [
    ("rtow", lambda: scenes.rtow_13_1(120, 75)[:2]),
    ("example_sdl", lambda: scenes.example_sdl(120, 75)),
    ("mesh", lambda: scenes.mesh_scene(96, 54, 24, 60)),
])
def test_glibc_libm_changes_little(oracle_lib, name, build):
    from oracle.binding import GLIBC_LIB_PATH, OracleScene
    cam, world = build()
    photo = cam.take_photo().samples(16).depth(16).seed(6)
    a, sa = OracleScene(world).render(cam.desc, photo.settings(), threads=8)
    b, sb = OracleScene(world, lib_path=GLIBC_LIB_PATH).render(cam.desc, photo.settings(), threads=8)
    d = a[..., :3].astype(np.float64) - b[..., :3].astype(np.float64)
    rmse = float(np.sqrt(np.mean(d * d)))
    same = float(np.mean(np.all(a == b, axis=-1)))
    assert rmse < 1e-4 and same > 0.95, (rmse, same)
