# dev: BVH2 vs BVH4 extend timing + parity on the bench frame
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
torch.cuda.set_device(0)
from raysnail_amd import scenes
from oracle.binding import OracleScene
res = {}
for tag, env in (("bvh2", "1"), ("bvh4", None)):
    if env: os.environ["RS_NO_BVH4"] = env
    cam, world, _, _ = scenes.rtow_13_1(800, 500)
    world.device_scene()
    os.environ.pop("RS_NO_BVH4", None)
    photo = cam.take_photo().samples(64).depth(8).seed(1)
    for _ in range(3):
        img = photo.shot(None, world); st = photo.last_stats
        print(f"{tag}: frame {st.ms:.2f} ms extend {st.kernel_ms:.2f} ms {st.samples/st.ms/1e3:.1f} Msamples/s segs {st.segments}", flush=True)
    res[tag] = img
print("bvh2 == bvh4 bitwise:", np.array_equal(res["bvh2"], res["bvh4"]))
cam, world, _, _ = scenes.rtow_13_1(200, 125)
photo = cam.take_photo().samples(16).depth(8).seed(1)
g = photo.shot(None, world)
r, _ = OracleScene(world).render(cam.desc, photo.settings(), threads=16)
print("bvh4 vs oracle exact:", np.array_equal(g, r))
