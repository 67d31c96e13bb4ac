# dev tool: parity + timing of megakernel vs wavefront (various chunk sizes) on the bench frame
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
torch.cuda.set_device(0)
from raysnail_amd import scenes
from oracle.binding import OracleScene

def render(mode, chunk=None, w=800, h=500, spp=64, reps=3, scene="rtow"):
    if chunk: os.environ["RS_WF_CHUNK"] = str(chunk)
    if scene == "rtow": cam, world, _, _ = scenes.rtow_13_1(w, h)
    else: cam, world = getattr(scenes, scene)(w, h)
    world.device_scene()
    os.environ.pop("RS_WF_CHUNK", None)
    photo = cam.take_photo().samples(spp).depth(8).seed(1).mode(mode)
    best = 1e9
    for _ in range(reps):
        img = photo.shot(None, world); st = photo.last_stats
        best = min(best, st.ms)
    return img, st, best, cam, world, photo

for scene, w, h in [("rtow", 200, 125), ("example_sdl", 160, 100), ("quadric_sdl", 128, 128), ("cornell_box", 100, 100)]:
    ref = None
    for mode in (1, 2):
        img, st, ms, cam, world, photo = render(mode, None, w, h, 16, 1, scene)
        if ref is None:
            ref, rs = OracleScene(world).render(cam.desc, photo.settings(), threads=16)
        d = np.abs(img[..., :3].astype(np.float64) - ref[..., :3])
        print(f"{scene} mode {mode}: exact={np.mean(np.all(img == ref, -1)):.4f} max={d.max():.2e} segs={st.segments} vs {rs.segments}", flush=True)

img1, st1, ms1, *_ = render(1)
print(f"mega: {ms1:.2f} ms  {st1.samples/ms1/1e3:.1f} Msamples/s kernel {st1.kernel_ms:.2f} ms", flush=True)
for chunk in (4 << 20, 26 << 20):
    img2, st2, ms2, *_ = render(2, chunk)
    print(f"wave chunk {chunk>>20}M: {ms2:.2f} ms  {st2.samples/ms2/1e3:.1f} Msamples/s extend {st2.kernel_ms:.2f} ms over {st2.kernel_launches} launches, "
          f"launches {st2.launches}, segs {st2.segments} == {st1.segments}: {st2.segments == st1.segments}, identical: {np.array_equal(img1, img2)}", flush=True)
