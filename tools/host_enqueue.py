# dev: host-side cost of enqueueing frames: time the asynchronous rs_render_device calls alone (no
# synchronisation) against the wall time until the GPU has finished them, for the bench frame and
# its N=8 row share. usage: python tools/host_enqueue.py [frames]
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.cuda.set_device(0)
from raysnail_amd import scenes
n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
cam, world, _, _ = scenes.rtow_13_1(800, 500)
photo = cam.take_photo().samples(64).depth(8).seed(1)
ds = world.device_scene()
ds.set_lanes(int(os.environ.get("RS_LANES", "2")))
fr = torch.zeros((500, 800, 4), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for rs in (1, 8):
    st = photo.rows(0, 0, rs).settings()
    for _ in range(5):
        ds.render_device(cam.desc, st, fr.data_ptr(), s, stats=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        ds.render_device(cam.desc, st, fr.data_ptr(), s, stats=False)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"rows 0::{rs}: enqueue {(t1 - t0) / n * 1e3:.3f} ms/frame, wall {(t2 - t0) / n * 1e3:.3f} ms/frame", flush=True)
