# quick GPU-vs-oracle probe used during development (not a test)
import sys, time, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import torch
torch.cuda.set_device(0)
from raysnail_amd import scenes
from oracle.binding import OracleScene
def cmp(name, cam, world, spp, depth):
    photo = cam.take_photo().samples(spp).depth(depth).seed(1)
    t = time.time(); gpu = photo.shot(None, world); tg = time.time() - t
    st = photo.last_stats
    t = time.time(); ref, rs = OracleScene(world).render(cam.desc, photo.settings(), threads=16); tc = time.time() - t
    d = np.abs(gpu[..., :3].astype(np.float64) - ref[..., :3])
    print(f"{name}: gpu {tg*1e3:.1f} ms (kernel {st.ms:.2f} ms) cpu {tc*1e3:.0f} ms  segs gpu={st.segments} cpu={rs.segments} "
          f"RMSE={np.sqrt((d**2).mean()):.3e} max={d.max():.3e} exact={np.mean(d.max(-1)==0):.4f} nan={np.isnan(gpu).sum()}", flush=True)
cam, world, _, _ = scenes.rtow_13_1(200, 125); cmp("rtow 200x125x16", cam, world, 16, 8)
cam, world = scenes.example_sdl(160, 100); cmp("example.sdl 160x100x16", cam, world, 16, 8)
cam, world = scenes.quadric_sdl(128, 128); cmp("quadric.sdl 128x128x16", cam, world, 16, 8)
cam, world = scenes.cornell_box(100, 100); cmp("cornell 100x100x16", cam, world, 16, 8)
cam, world, _, _ = scenes.rtow_13_1(800, 500)
photo = cam.take_photo().samples(64).depth(8).seed(1)
for i in range(3):
    t = time.time(); img = photo.shot(None, world); dt = time.time() - t
    st = photo.last_stats
    print(f"rtow 800x500x64: {dt*1e3:.1f} ms host, {st.ms:.1f} ms in-call, {st.samples/st.ms/1e3:.1f} Msamples/s, segs/sample {st.segments/st.samples:.3f}", flush=True)
