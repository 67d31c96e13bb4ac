# dev: K row-share frames (rows 0::8 of the bench frame) one lane, one frame slot, for rocprofv3 kernel traces of
# the one-call-per-pass frames against rs_render_device_passes' sample stream.  usage: passes_trace.py single|stream [K] [row_step]
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.cuda.set_device(0)
from raysnail_amd import scenes
mode = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 12
rs = int(sys.argv[3]) if len(sys.argv) > 3 else 8
cam, world, _, _ = scenes.rtow_13_1(800, 500)
photo = cam.take_photo().samples(64).depth(8).seed(1)
ds = world.device_scene()
ds.set_lanes(1)
ds.set_frames_in_flight(1)
frame = torch.zeros((500, 800, 4), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for rep in range(2):  # the second repetition is the one to read
    if mode == "single":
        for k in range(K):
            ds.render_device(cam.desc, photo.rows(0, 0, rs).pass_index(k).settings(), frame.data_ptr(), s, stats=False)
    else:
        ds.render_device_passes(cam.desc, photo.rows(0, 0, rs).pass_index(0).settings(), [frame.data_ptr()] * K, s,
                                stats=False)
    torch.cuda.synchronize()
print("done", flush=True)
