# dev: first diverging bounce of one sample (GPU rs_probe_samples vs oracle), then a world-hit
# comparison on every ray of the oracle's path
import ctypes as C, os, re, sys, tempfile
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
torch.cuda.set_device(0)
from raysnail_amd import scenes
from oracle.binding import OracleScene
x, y, spp, s = map(int, sys.argv[1:5])
cam, world = scenes.mesh_scene(1920, 1080)
ds = world.device_scene()
orc = OracleScene(world)
orc.lib.orc_set_trace.argtypes = [C.c_int]
def both(depth):
    st = cam.take_photo().samples(spp).depth(depth).seed(1).settings()
    g = np.zeros((1, 4))
    assert ds.lib.rs_probe_samples(ds.handle, C.byref(cam.desc), C.byref(st), x, y, s, 1, g.ctypes.data) == 0
    o = (C.c_double * 3)(); seg = C.c_uint64()
    orc.lib.orc_sample_radiance(orc.h, C.byref(cam.desc), C.byref(st), x, y, s, o, C.byref(seg))
    return g[0], np.array(o[:]), seg.value, st
first = None
for d in range(1, 51):
    g, o, seg, st = both(d)
    if not (np.array_equal(g[:3], o) and g[3] == seg):
        first = d
        print("first divergence at depth", d, "gpu", g, "oracle", o, seg)
        break
if first is None:
    print("no divergence"); sys.exit(0)
# oracle trace of that depth
fd = tempfile.TemporaryFile(mode="w+")
old = os.dup(2); os.dup2(fd.fileno(), 2)
orc.lib.orc_set_trace(1)
o = (C.c_double * 3)(); seg = C.c_uint64()
orc.lib.orc_sample_radiance(orc.h, C.byref(cam.desc), C.byref(st), x, y, s, o, C.byref(seg))
orc.lib.orc_set_trace(0)
os.dup2(old, 2); fd.seek(0)
lines = [l for l in fd.read().splitlines() if l.startswith("depth")]
num = r"(-?[0-9.e+\-]+|-?nan|-?inf)"
for l in lines[-4:]:
    print(l)
for l in lines:
    m = re.match(r"depth (\d+) o \((\S+) (\S+) (\S+)\) d \((\S+) (\S+) (\S+)\)", l)
    oo = np.array([float(m.group(i)) for i in (2, 3, 4)]); dd = np.array([float(m.group(i)) for i in (5, 6, 7)])
    rays = np.ascontiguousarray(np.concatenate([oo, dd, [0.0]])[None])
    out = np.zeros((1, 13))
    ds.lib.rs_probe_world_hit(ds.handle, rays.ctypes.data, 1, 1e-4, float("inf"), out.ctypes.data)
    r = np.array(orc.world_hit(oo, dd))
    same = r[0] == out[0, 0] and (r[0] == 0 or (np.array_equal(r[1:9], out[0, 1:9]) and r[11] == out[0, 11]))
    if not same:
        print("WORLD-HIT MISMATCH at", m.group(1), "gpu", out[0, :9], "oracle", r[:9])
print("checked", len(lines), "levels")
