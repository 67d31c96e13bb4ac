# dev: per-sample GPU vs oracle radiance for one pixel (rs_probe_samples / orc_sample_radiance)
import ctypes as C, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
torch.cuda.set_device(0)
from raysnail_amd import scenes
from oracle.binding import OracleScene
x, y, spp, depth = map(int, sys.argv[1:5])
cam, world = scenes.mesh_scene(1920, 1080)
photo = cam.take_photo().samples(spp).depth(depth).seed(1)
st = photo.settings()
ds = world.device_scene()
n = int(spp ** 0.5) ** 2
g = np.zeros((n, 4))
assert ds.lib.rs_probe_samples(ds.handle, C.byref(cam.desc), C.byref(st), x, y, 0, n, g.ctypes.data) == 0, ds.lib.rs_last_error()
orc = OracleScene(world)
for s in range(n):
    o = (C.c_double * 3)(); seg = C.c_uint64()
    orc.lib.orc_sample_radiance(orc.h, C.byref(cam.desc), C.byref(st), x, y, s, o, C.byref(seg))
    if not (np.array_equal(g[s, :3], np.array(o[:])) and g[s, 3] == seg.value):
        print("sample", s, "gpu", g[s], "oracle", o[:], seg.value)
print("done")
