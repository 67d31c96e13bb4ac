# dev: locate GPU-vs-oracle differences on the C5 mesh scene
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
torch.cuda.set_device(0)
from raysnail_amd import scenes
from oracle.binding import OracleScene
spp, depth, step = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
cam, world = scenes.mesh_scene(1920, 1080)
photo = cam.take_photo().samples(spp).depth(depth).seed(1)
img = photo.shot(None, world)
orc = OracleScene(world)
ref, _ = orc.render(cam.desc, photo.rows(0, 0, step).settings(), threads=16)
g, r = img[::step], ref[::step]
bad = np.argwhere(np.any(g != r, axis=-1))
print("rows", g.shape[0], "bad pixels", len(bad), "nan gpu", int(np.isnan(g).any(-1).sum()), "nan ref", int(np.isnan(r).any(-1).sum()))
for (y, x) in bad[:10]:
    print((y * step, x), g[y, x], r[y, x])
# world-hit probe of random rays from the camera region
ds = world.device_scene()
rng = np.random.default_rng(1)
n = 20000
eye = np.array(cam.desc.look_from[:])
o = eye + rng.normal(0, 0.3, (n, 3))
tgt = np.array([0.0, 0.9, 0.0]) + rng.normal(0, 0.7, (n, 3))
d = tgt - o
d /= np.linalg.norm(d, axis=1, keepdims=True)
rays = np.ascontiguousarray(np.concatenate([o, d, np.zeros((n, 1))], 1))
out = np.zeros((n, 13))
assert ds.lib.rs_probe_world_hit(ds.handle, rays.ctypes.data, n, 1e-4, float("inf"), out.ctypes.data) == 0
nb = 0
for i in range(n):
    rr = np.array(orc.world_hit(o[i], d[i]))
    gg = out[i]
    same = rr[0] == gg[0] and (rr[0] == 0 or (np.array_equal(rr[1:9], gg[1:9]) and rr[11] == gg[11] and rr[12] == gg[12]))
    if not same:
        nb += 1
        if nb <= 5:
            print("hit mismatch", i, "gpu", gg[:9], "orc", rr[:9])
print("world-hit mismatches", nb, "of", n)
