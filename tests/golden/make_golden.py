"""Regenerate the golden fixtures of tests/golden/ from the CPU oracle (oracle/oracle.cpp).

The reference (Rust) cannot be built or run in this container (no cargo/rustc, no crate sources),
so these fixtures are produced by the restatement; they pin the restatement against regressions
and give the GPU tests a fixed target. Published third-party vectors are recorded alongside.
Run: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle.binding import OracleScene  # noqa: E402
from raysnail_amd import scenes  # noqa: E402
from raysnail_amd.api import Sphere  # noqa: E402

FRAMES = {
    # name: (builder, kwargs, spp, depth, seed)
    "rtow": (lambda: scenes.rtow_13_1(48, 30)[:2], 16, 8, 1),
    "example_sdl": (lambda: scenes.example_sdl(48, 30), 16, 8, 1),
    "quadric_sdl": (lambda: scenes.quadric_sdl(48, 48), 16, 8, 1),
    "cornell": (lambda: scenes.cornell_box(40, 40), 16, 8, 1),
    "rtow_depth50": (lambda: scenes.rtow_13_1(32, 20)[:2], 9, 50, 3),
    # BASELINE config C1 exactly: examples/rtow_13_1.rs's scene at 400x225, 16 spp, depth 8
    "rtow_c1": (lambda: scenes.rtow_13_1(400, 225)[:2], 16, 8, 1),
}


def render_frame(name):
    build, spp, depth, seed = FRAMES[name]
    cam, world = build()
    photo = cam.take_photo().samples(spp).depth(depth).seed(seed)
    img, stats = OracleScene(world).render(cam.desc, photo.settings(), threads=8)
    return img, stats


def rtow_scene_digest(seed=7):
    lst = scenes.balls_scene(seed, True)
    spheres = [o for o in lst.objects if isinstance(o, Sphere)]
    kinds = {}
    h = hashlib.sha256()
    for s in spheres:
        k = type(s.material).__name__
        kinds[k] = kinds.get(k, 0) + 1
        h.update(np.array(list(s.center) + [s.radius], dtype=np.float64).tobytes())
        h.update(k.encode())
    return {"n_objects": len(lst.objects), "kinds": kinds, "sha256": h.hexdigest(),
            "first": [list(s.center) + [s.radius] for s in spheres[1:6]]}


def main():
    frames = {}
    meta = {}
    for name in FRAMES:
        img, st = render_frame(name)
        frames[name] = img
        meta[name] = {"samples": int(st.samples), "segments": int(st.segments)}
        print(name, img.shape, meta[name])
    np.savez_compressed(os.path.join(HERE, "oracle_frames.npz"), **frames)
    kat = {
        "xorshift128_marsaglia": {"seed_words": [123456789, 362436069, 521288629, 88675123],
                                  "u32": [3701687786, 458299110, 2500872618, 3633119408, 516391518, 2377269574],
                                  "source": "Marsaglia 2003, xor128 (published sequence)"},
        "rand_xorshift_true_values": {"seed_bytes": list(range(16, 0, -1)),
                                      "u32": [2081028795, 620940381, 269070770, 16943764, 854422573, 29242889,
                                              1550291885, 1227154591, 271695242],
                                      "source": "rand_xorshift 0.3.0 tests::test_xorshift_true_values"},
        "chacha20_rfc7539_2_3_2": {"key": "000102...1f", "counter": 1, "nonce": "000000090000004a00000000",
                                   "words": ["e4e7f110", "15593bd1", "1fdd0f50", "c47120a3", "c7f4d1c7", "0368c033",
                                             "9aaa2204", "4e6cd4c3", "466482d2", "09aa9f07", "05d7c214", "a2028bd9",
                                             "d19c12b5", "b94e16de", "e883d0cb", "4e3c50a2"],
                                   "source": "RFC 7539 section 2.3.2"},
        "frames": meta,
        "rtow_seed7_scene": rtow_scene_digest(7),
    }
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)


if __name__ == "__main__":
    main()
