# dev: one depth-50 SDL frame against the oracle (tests/test_gpu_configs.py::test_sdl_scenes_depth50 alone), for
# isolating a failure. usage: python tools/repro_depth50.py <example_sdl|quadric_sdl> [spp] [lib.so]
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from raysnail_amd import _abi
if len(sys.argv) > 3:
    _abi.lib_path = lambda: sys.argv[3]
import numpy as np
import torch
torch.cuda.set_device(0)
from raysnail_amd import scenes
from oracle.binding import OracleScene
name = sys.argv[1]
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 4
cam, world = {"example_sdl": lambda: scenes.example_sdl(64, 40), "quadric_sdl": lambda: scenes.quadric_sdl(48, 48)}[name]()
photo = cam.take_photo().samples(spp).depth(50).seed(21)
img = photo.shot(None, world)
print("gpu segments", photo.last_stats.segments, flush=True)
ref, rs = OracleScene(world).render(cam.desc, photo.settings(), threads=16)
print("oracle segments", rs.segments, "identical pixels", float(np.mean(np.all(img == ref, axis=-1))), flush=True)
