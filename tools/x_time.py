# dev: time the rich-mode scenes (X1 all_feature_scene, X2 cornell_smoke) with the package of any
# tree (a git worktree of an earlier commit, built in place): best of 3 frames after a warm-up.
# usage: python tools/x_time.py <tree root> [x1|x2 ...]
import hashlib, os, sys, time
root = os.path.abspath(sys.argv[1])
sys.path.insert(0, root)
import torch
torch.cuda.set_device(0)
from raysnail_amd import scenes
SC = {"x1": (lambda: scenes.all_feature_scene(400, 400), 16, 50), "x2": (lambda: scenes.cornell_smoke(300, 300), 64, 50)}
for key in sys.argv[2:] or ["x1", "x2"]:
    mk, spp, depth = SC[key]
    cam, world = mk()[:2]
    photo = cam.take_photo().samples(spp).depth(depth).seed(1)
    img = photo.shot(None, world)
    best = None
    for _ in range(3):
        t0 = time.perf_counter(); img = photo.shot(None, world); dt = time.perf_counter() - t0
        best = dt if best is None or dt < best else best
    print(f"{os.path.basename(root)} {key}: {best * 1e3:.2f} ms md5 {hashlib.md5(img.tobytes()).hexdigest()[:12]}", flush=True)
