# dev: render rows 0::K of the bench frame (one rank's share at N = K) `reps` times into a device
# buffer, for rocprofv3 kernel traces of the N = K per-GPU workload.  usage: share_frames.py [K] [reps]
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.cuda.set_device(0)
from raysnail_amd import scenes
K = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
cam, world, _, _ = scenes.rtow_13_1(800, 500)
photo = cam.take_photo().samples(64).depth(8).seed(1)
ds = world.device_scene()
frame = torch.zeros((500, 800, 4), dtype=torch.float32, device="cuda")
st = photo.rows(0, 0, K).settings()
for i in range(reps + 2):
    if i == 2:
        torch.cuda.synchronize(); t0 = time.perf_counter()
    ds.render_device(cam.desc, st, frame.data_ptr(), torch.cuda.current_stream().cuda_stream, stats=False)
torch.cuda.synchronize()
print(f"rows 0::{K}: {(time.perf_counter() - t0) / reps * 1e3:.3f} ms per share frame", flush=True)
