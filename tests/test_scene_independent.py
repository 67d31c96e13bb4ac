"""The RTIOW scene has two independent builders: raysnail_amd/scenes.py (Python, feeds the GPU) and
oracle/scene_gen.cpp (C++, the oracle's own). Both restate examples/common/scene.rs:23-191 over
rand 0.8.3's StdRng (ChaCha12) and UniformFloat; they must agree sphere for sphere and with the
committed digest (tests/golden/kat.json), so a mis-restated scene cannot hide behind a shared
generator in the GPU-vs-oracle frame tests."""
import hashlib
import json
import os

import numpy as np
import pytest

from raysnail_amd import scenes
from raysnail_amd.api import Dielectric, DiffuseMetal, Lambertian, Metal, Sphere
from raysnail_amd import _abi as A

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
KIND_NAMES = {A.RS_MAT_LAMBERTIAN: "Lambertian", A.RS_MAT_METAL: "Metal", A.RS_MAT_DIFFUSE_METAL: "DiffuseMetal",
              A.RS_MAT_DIELECTRIC: "Dielectric"}


def _kat():
    return json.load(open(os.path.join(GOLDEN, "kat.json")))


def test_cpp_chacha_core_matches_rfc7539():
    """RFC 7539 section 2.3.2 block (20 rounds) through the C++ core the oracle's StdRng uses."""
    import ctypes as C
    from oracle.binding import load
    v = _kat()["chacha20_rfc7539_2_3_2"]
    key = bytes.fromhex("".join(f"{i:02x}" for i in range(32)))
    nonce = bytes.fromhex(v["nonce"])
    st = [0x61707865, 0x3320646e, 0x79622d32, 0x6b206574]
    st += [int.from_bytes(key[4 * i:4 * i + 4], "little") for i in range(8)]
    st += [v["counter"]] + [int.from_bytes(nonce[4 * i:4 * i + 4], "little") for i in range(3)]
    out = (C.c_uint32 * 16)()
    load().orc_chacha_block((C.c_uint32 * 16)(*st), 20, out)
    assert [f"{w:08x}" for w in out] == v["words"]


def test_cpp_scene_equals_python_scene():
    from oracle.binding import rtow_balls
    cpp = rtow_balls(7)
    py = [o for o in scenes.balls_scene(7, True).objects]
    assert len(py) == cpp.shape[0] == _kat()["rtow_seed7_scene"]["n_objects"]
    for row, s in zip(cpp, py):
        assert isinstance(s, Sphere)
        assert tuple(row[:3]) == tuple(s.center) and row[3] == s.radius
        m = s.material
        kind = {Lambertian: A.RS_MAT_LAMBERTIAN, Metal: A.RS_MAT_METAL, DiffuseMetal: A.RS_MAT_DIFFUSE_METAL,
                Dielectric: A.RS_MAT_DIELECTRIC}[type(m)]
        assert int(row[4]) == kind
        if int(row[5]):        # the checker ground
            continue
        col = m.color if isinstance(m, Dielectric) else m.texture
        assert np.array_equal(np.float32(row[6:9]), np.float32([col.r, col.g, col.b]))  # the ABI takes f32
        if kind == A.RS_MAT_DIFFUSE_METAL:
            assert row[9] == m.exponent
        if kind == A.RS_MAT_DIELECTRIC:
            assert row[9] == m.refractive and m.glass


def test_cpp_scene_matches_committed_digest():
    from oracle.binding import rtow_balls
    cpp = rtow_balls(7)
    h = hashlib.sha256()
    kinds = {}
    for row in cpp:
        name = KIND_NAMES[int(row[4])]
        kinds[name] = kinds.get(name, 0) + 1
        h.update(np.array(row[:4], dtype=np.float64).tobytes())
        h.update(name.encode())
    ref = _kat()["rtow_seed7_scene"]
    assert h.hexdigest() == ref["sha256"]
    assert kinds == ref["kinds"]


def test_oracle_frames_from_both_builders_agree():
    from oracle.binding import OracleScene
    cam, world, _, _ = scenes.rtow_13_1(48, 30)
    st = cam.take_photo().samples(4).depth(8).seed(3).settings()
    a, sa = OracleScene(world).render(cam.desc, st, threads=8)
    b, sb = OracleScene(rtow_seed=7).render(cam.desc, st, threads=8)
    assert sa.segments == sb.segments
    assert np.array_equal(a, b)


@pytest.mark.gpu
def test_gpu_frame_against_independently_built_oracle_scene(gpu):
    """GPU (scene from scenes.py) vs oracle (scene from scene_gen.cpp) on RTIOW seed 7."""
    from oracle.binding import OracleScene
    cam, world, _, _ = scenes.rtow_13_1(96, 60)
    photo = cam.take_photo().samples(16).depth(8).seed(11)
    img = photo.shot(None, world)
    ref, rs = OracleScene(rtow_seed=7).render(cam.desc, photo.settings(), threads=16)
    assert photo.last_stats.segments == rs.segments
    d = np.abs(img[..., :3].astype(np.float64) - ref[..., :3].astype(np.float64))
    assert float(np.sqrt(np.mean(d * d))) < 1e-4
    assert np.mean(np.all(img == ref, axis=-1)) >= 0.999
