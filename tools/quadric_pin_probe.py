# dev: render sdl/quadric.sdl the CLI's way (800x500, 122 -> 121 spp, depth 8, one pass) on the GPU and
# compare block means with the reference's own render (tests/golden/sdl_quadrics_pin.json)
import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch; torch.cuda.set_device(0)
from raysnail_amd import scenes
pin = json.load(open(os.path.join(ROOT, "tests/golden/sdl_quadrics_pin.json")))
B = pin["block"]
ref_m = np.array(pin["block_mean"]); ref_s = np.array(pin["block_std"])
for spp, depth, seed in ((122, 8, 1), (122, 8, 2), (122, 50, 1)):
    cam, world = scenes.quadric_sdl(800, 500, cornell_emitter=False)
    img = cam.take_photo().samples(spp).depth(depth).seed(seed).shot(None, world)
    q = np.floor(np.clip(img[..., :3].astype(np.float64), 0.0, 1.0) * 255.5).clip(0, 255) / 255.0
    h, w = q.shape[:2]
    m = q[: h // B * B, : w // B * B].reshape(h // B, B, w // B, B, 3).mean(axis=(1, 3))
    d = np.abs(m - ref_m)
    print(json.dumps({"spp": spp, "depth": depth, "seed": seed, "global_mean": q.mean(axis=(0, 1)).round(5).tolist(),
                      "ref_global": pin["global_mean_rgb"], "block_absdiff_mean": round(float(d.mean()), 5),
                      "block_absdiff_p95": round(float(np.percentile(d, 95)), 5),
                      "block_absdiff_max": round(float(d.max()), 5),
                      "frac_blocks_within_0.02": round(float(np.mean(d.max(-1) < 0.02)), 4),
                      "worst_blocks": [list(map(int, np.unravel_index(i, d.max(-1).shape))) for i in np.argsort(-d.max(-1).ravel())[:8]]}),
          flush=True)
    np.save(os.path.join(ROOT, "gpurun_out", f"quadric_cli_{spp}_{depth}_{seed}.npy"), (q * 255).round().astype(np.uint8))
