# dev: time one frame of a named scene with a given libraysnail_hip build (variants from tools/build_variant.sh)
# usage: python tools/time_scene.py <lib.so|default> <scene> [spp] [depth] [WxH]
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from raysnail_amd import _abi
if sys.argv[1] != "default":
    _abi.lib_path = lambda: sys.argv[1]
import torch; torch.cuda.set_device(0)
from raysnail_amd import scenes
name = sys.argv[2]
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 16
depth = int(sys.argv[4]) if len(sys.argv) > 4 else 50
W, H = map(int, (sys.argv[5] if len(sys.argv) > 5 else "960x540").split("x"))
def mesh_inside():
    """C5's mesh seen from inside (every ray is an interior one, like C5's trapped paths)"""
    from raysnail_amd.api import CameraBuilder
    _, world = scenes.mesh_scene(W, H)
    cam = CameraBuilder().look_from((0.0, 1.0, 0.0)).look_at((1.0, 1.0, 0.3)).fov(60.0).width(W).height(H).build()
    return cam, world
build = {"mesh": lambda: scenes.mesh_scene(W, H), "rtow": lambda: scenes.rtow_13_1(W, H)[:2], "mesh_in": mesh_inside,
         "quadric": lambda: scenes.quadric_sdl(W, H), "example": lambda: scenes.example_sdl(W, H),
         "all_feature": lambda: scenes.all_feature_scene(W, H), "smoke": lambda: scenes.cornell_smoke(W, H),
         "deep": lambda: scenes.deep_spheres(W, H)}[name]
cam, world = build()
photo = cam.take_photo().samples(spp).depth(depth).seed(1)
photo.shot(None, world)
best = None
for _ in range(3):
    t0 = time.perf_counter(); img = photo.shot(None, world); dt = time.perf_counter() - t0
    best = dt if best is None or dt < best else best
st = photo.last_stats
print(json.dumps({"lib": os.path.basename(sys.argv[1]), "scene": name, "ms": round(best * 1e3, 2),
                  "kernel_ms": round(st.kernel_ms, 2), "Gseg_s": round(st.segments / best / 1e9, 3),
                  "seg_per_sample": round(st.segments / st.samples, 3), "tree": st.tree_arity,
                  "checksum": float(img[..., :3].astype("float64").sum())}), flush=True)
