# dev: C4 frame timings in the ways tools/bench_configs.py and tools/time_scene.py take them (host-output frames with
# statistics, asynchronous device frames), for one library.  usage: python tools/c4_diag.py <lib.so|default> [spp]
import os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from raysnail_amd import _abi
if sys.argv[1] != "default":
    _abi.lib_path = lambda: sys.argv[1]
import torch; torch.cuda.set_device(0)
from raysnail_amd import scenes
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
cam, world = scenes.quadric_sdl(1024, 1024)
ds = world.device_scene()
photo = cam.take_photo().samples(spp).depth(50).seed(1)
out = {"lib": os.path.basename(sys.argv[1])}
for k in range(2):
    t0 = time.perf_counter(); photo.shot(None, world); out[f"host{k}_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
    out[f"host{k}_launches"] = photo.last_stats.launches
frame = torch.zeros((1024, 1024, 4), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for k in range(4):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    ds.render_device(cam.desc, photo.settings(), frame.data_ptr(), s, stats=False)
    torch.cuda.synchronize(); out[f"dev{k}_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
st = ds.render_device(cam.desc, photo.settings(), frame.data_ptr(), s, stats=True)
out["dev_stats_launches"] = st.launches
out["dev_stats_ms"] = round(st.ms, 1)
print(json.dumps(out), flush=True)
