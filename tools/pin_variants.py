# dev: which semantics reproduce the reference's own render (examples/sdl_quadrics.jpg)?
# Renders sdl/quadric.sdl the CLI's way with the CPU oracle under each diagnostic variant
# (oracle.cpp ORC_VAR_*) and reports per-block z-scores against the pin (tests/pinlib.py).
# Output: one JSON line per variant (profiles/r3/pin_variants.jsonl).
#   python tools/pin_variants.py [spp] [out.jsonl]
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import pinlib
from raysnail_amd import scenes
from oracle import binding as ob

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 49
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "r3", "pin_variants.jsonl")
os.makedirs(os.path.dirname(out), exist_ok=True)
names = {0: "checkout semantics", ob.VAR_LIGHT_RADIUS: "Sphere::random scaled by the radius",
         ob.VAR_LIGHT_FROM_POINT: "light ray from hit.point", ob.VAR_SORTED_ROOTS: "quadric roots smaller first",
         ob.VAR_RECT_CLOSED_END: "AARect accepts t == range end", ob.VAR_TREE_FILE_ORDER: "BVH in file order"}
runs = [(0, 0), (ob.VAR_LIGHT_RADIUS, 0), (ob.VAR_LIGHT_FROM_POINT, 0), (ob.VAR_SORTED_ROOTS, 0)]
runs += [(ob.VAR_REF_TREE, a) for a in range(8)]
runs += [(ob.VAR_RECT_CLOSED_END, 0), (ob.VAR_TREE_FILE_ORDER, 0)]
p = pinlib.pin()
with open(out, "w") as f:
    for bits, axes in runs:
        t = time.time()
        with ob.variant(bits, axes):
            cam, world = scenes.quadric_sdl(800, 500, cornell_emitter=False)
            img, _ = ob.OracleScene(world).render(cam.desc, cam.take_photo().samples(spp).depth(8).seed(3).settings(),
                                                  threads=os.cpu_count() or 4)
        q = pinlib.quantize(img)
        z = pinlib.zmap(q, spp, p=p)
        az = np.abs(z).max(-1)
        worst = np.argsort(-az.ravel())[:5]
        rec = {"variant": bits, "axis_bits": axes,
               "what": names.get(bits, "bvh.rs tree, Random::range(0..2) draws = %d%d%d (preorder)" % (axes & 1, axes >> 1 & 1, axes >> 2 & 1)),
               "spp": spp, "seed": 3, "max_abs_z": round(float(az.max()), 2), "blocks_z_ge_4.5": int((az >= 4.5).sum()),
               "z_block_7_12": np.round(z[7, 12], 2).tolist(), "z_block_6_26": np.round(z[6, 26], 2).tolist(),
               "worst_blocks": [[int(i // az.shape[1]), int(i % az.shape[1]), round(float(az.ravel()[i]), 2)] for i in worst],
               "global_gap": np.round(pinlib.global_gap(q, p), 4).tolist(), "seconds": round(time.time() - t, 1)}
        print(json.dumps(rec), flush=True)
        f.write(json.dumps(rec) + "\n")
