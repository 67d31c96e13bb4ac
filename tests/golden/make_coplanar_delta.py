"""Generate tests/golden/sdl_quadrics_coplanar_delta.json: the per-block effect of the one semantic
difference between the reference checkout and the code that rendered examples/sdl_quadrics.jpg.

Finding (tools/pin_variants.py). In sdl/quadric.sdl the floor box's top face (y = -1,
`box { <-3.5, -1.2, -8>, <3.5, -1, 6> }`) is coplanar with the bottom faces of the clipping boxes of
the cone (`translate <-1, 0, 2>`) and the hyperboloid (`translate <-1, 0, -4>`). Every tree that the
checkout's BVH::new can build (bvh.rs:58-113: Random::range(0..2) axes, sort by bbox min) visits the
floor box before those two objects, so BVH::hit (bvh.rs:173-192) hands them the range
[1e-4, t_floor). A ray that starts inside the clipping box -- from the underside of the upper cone
towards the lower cone, or across the hyperboloid's waist -- reaches the quadric before the floor,
but the clipping box's only face hit (its exit through the bottom, at exactly t_floor) is outside
the half-open range (rect.rs:102), Box::hit returns None and Intersection::hit (intersection.rs:63)
needs both children: the lower cone is missed and the floor behind it is returned. The reference's
JPEG shows that surface lit (the underside of the upper cone ~0.05 brighter near the waist).

The oracle with ORC_VAR_RECT_CLOSED_END (AARect accepts t == range end) -- or, equally, with the
objects visited in file order (ORC_VAR_TREE_FILE_ORDER) -- matches all 640 blocks of the JPEG
within Monte Carlo noise (max |z| ~2.2); with the checkout's semantics 10 blocks, all on those two
objects, are 4-24 sigma off. This file stores, per block, (variant - checkout) block means of the
quantised oracle frames rendered at the GPU test's exact settings (800x500, 122 -> 121 spp, depth
8, seed 1), so the GPU test adds the proven effect and then compares every block with budget 0.

usage: python tests/golden/make_coplanar_delta.py   (~40 s on 8 cores)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

SPP, DEPTH, SEED = 122, 8, 1


def render(bits, spp=SPP, seed=SEED, threads=0):
    from oracle.binding import OracleScene, variant
    from raysnail_amd import scenes
    with variant(bits):
        cam, world = scenes.quadric_sdl(800, 500, cornell_emitter=False)
        img, _ = OracleScene(world).render(cam.desc, cam.take_photo().samples(spp).depth(DEPTH).seed(seed).settings(),
                                           threads=threads or (os.cpu_count() or 4))
    return img


def main():
    import pinlib
    from oracle.binding import VAR_RECT_CLOSED_END
    B = pinlib.pin()["block"]
    base = pinlib.block_means(pinlib.quantize(render(0)), B)
    var = pinlib.block_means(pinlib.quantize(render(VAR_RECT_CLOSED_END)), B)
    delta = var - base
    out = {
        "what": "block means of quantised oracle frames, ORC_VAR_RECT_CLOSED_END minus the checkout's semantics",
        "settings": {"width": 800, "height": 500, "spp": SPP, "depth": DEPTH, "seed": SEED},
        "block": B,
        "delta": np.round(delta, 6).tolist(),
    }
    with open(os.path.join(HERE, "sdl_quadrics_coplanar_delta.json"), "w") as f:
        json.dump(out, f)
    moved = np.argwhere(np.abs(delta).max(-1) > 0.002)
    print("blocks moved by > 0.002:", [tuple(map(int, b)) for b in moved])


if __name__ == "__main__":
    main()
