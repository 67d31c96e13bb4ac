import sys, numpy as np, ctypes as C
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import torch; torch.cuda.set_device(0)
from raysnail_amd import scenes, _abi as A
from oracle.binding import OracleScene
cam, world = scenes.quadric_sdl(128, 128)
ds = world.device_scene(); orc = OracleScene(world)
rng = np.random.default_rng(0)
n = 200000
o = rng.uniform(-6, 6, (n, 3)); o[:, 1] = rng.uniform(-1.5, 4, n)
d = rng.standard_normal((n, 3)); d /= np.linalg.norm(d, axis=1, keepdims=True)
rays = np.concatenate([o, d, np.zeros((n, 1))], 1).copy()
out = np.zeros((n, 13))
rc = ds.lib.rs_probe_world_hit(ds.handle, rays.ctypes.data, n, 1e-4, float('inf'), out.ctypes.data)
assert rc == 0, ds.lib.rs_last_error()
bad = 0
for i in range(n):
    r = orc.world_hit(o[i], d[i])
    g = out[i]
    ok = (r[0] == g[0]) and (r[0] == 0 or (r[1] == g[1] and r[2] == g[2] and r[3:9] == list(g[3:9]) and r[11] == g[11] and r[12] == g[12]))
    if not ok:
        bad += 1
        if bad <= 8:
            print("ray", i, o[i].tolist(), d[i].tolist()); print(" cpu", r); print(" gpu", g.tolist())
print("mismatches", bad, "of", n)
