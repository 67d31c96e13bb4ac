# dev: what rank 0's row gather costs on top of the N = K row-share frames (bench.py row_share), op by op:
# the share loop alone, + the pack copy, + the receive-buffer copy, + the de-interleave, each pipelined like the
# bench loop.  usage: python tools/gather_probe.py [K] [steps]
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.cuda.set_device(0)
from raysnail_amd import scenes

K = int(sys.argv[1]) if len(sys.argv) > 1 else 8
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cam, world, _, _ = scenes.rtow_13_1(800, 500)
photo = cam.take_photo().samples(64).depth(8).seed(1)
ds = world.device_scene()
H, W = 500, 800
frame = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
st = photo.rows(0, 0, K).settings()
per = (H + K - 1) // K
n = len(range(0, H, K))
packed = torch.zeros((per, W, 4), dtype=torch.float32, device="cuda")
allp = torch.zeros((K, per, W, 4), dtype=torch.float32, device="cuda")
src = torch.zeros_like(allp)
full = torch.empty((per * K, W, 4), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream().cuda_stream


def step(level):
    ds.render_device(cam.desc, st, frame.data_ptr(), s, stats=False)
    if level >= 1:
        packed[:n].copy_(frame[0::K])
    if level >= 2:
        allp.copy_(src)
    if level >= 3:
        full.view((per, K, W, 4)).copy_(allp.transpose(0, 1))


names = ["share alone", "+ pack copy", "+ receive copy", "+ de-interleave"]
res = {}
for rep in range(2):
    for level in range(4):
        for _ in range(5):
            step(level)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step(level)
        torch.cuda.synchronize()
        res.setdefault(level, []).append((time.perf_counter() - t0) / steps * 1e3)
for level in range(4):
    print(f"{names[level]:18s} {min(res[level]):.4f} ms per share frame", flush=True)
# the copies alone, the GPU otherwise idle
for level, fn in ((1, lambda: packed[:n].copy_(frame[0::K])), (2, lambda: allp.copy_(src)),
                  (3, lambda: full.view((per, K, W, 4)).copy_(allp.transpose(0, 1)))):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100):
        fn()
    e1.record(); torch.cuda.synchronize()
    print(f"{names[level][2:]:16s} alone: {e0.elapsed_time(e1) / 100 * 1e3:.1f} us", flush=True)
