# renders the bench frame a few times (for profilers); args: mode reps [scene spp depth]
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
torch.cuda.set_device(0)
from raysnail_amd import scenes
mode = int(sys.argv[1]) if len(sys.argv) > 1 else 0
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
scene = sys.argv[3] if len(sys.argv) > 3 else "rtow"
spp = int(sys.argv[4]) if len(sys.argv) > 4 else 64
depth = int(sys.argv[5]) if len(sys.argv) > 5 else 8
if scene == "rtow":
    cam, world, _, _ = scenes.rtow_13_1(800, 500)
else:
    cam, world = getattr(scenes, scene)(800, 500)
photo = cam.take_photo().samples(spp).depth(depth).seed(1).mode(mode)
for _ in range(reps):
    photo.shot(None, world)
    st = photo.last_stats
    print(f"{st.ms:.2f} ms kernel {st.kernel_ms:.2f} ms segs {st.segments}", flush=True)
