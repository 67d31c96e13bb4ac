# dev: host time of enqueueing frames (asynchronous rs_render_device calls, no synchronisation inside the loop)
# against the wall time until the GPU has run them, for the bench frame and its N = 8 row share; and the same with
# the settings built once instead of per call. usage: python tools/host_probe.py [frames]
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.cuda.set_device(0)
from raysnail_amd import scenes
n = int(sys.argv[1]) if len(sys.argv) > 1 else 30
cam, world, _, _ = scenes.rtow_13_1(800, 500)
photo = cam.take_photo().samples(64).depth(8).seed(1)
ds = world.device_scene()
frame = torch.zeros((500, 800, 4), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for K in (1, 8):
    st = photo.rows(0, 0, K).settings()
    for _ in range(5):
        ds.render_device(cam.desc, st, frame.data_ptr(), s, stats=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        ds.render_device(cam.desc, st, frame.data_ptr(), s, stats=False)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"rows 0::{K}: host enqueue {(t1 - t0) / n * 1e3:.3f} ms per frame, wall {(t2 - t0) / n * 1e3:.3f} ms per frame",
          flush=True)
