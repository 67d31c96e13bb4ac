# DIAGNOSTIC: time extend with the ablated-leaf library (results intentionally wrong)
import os, sys, ctypes
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raysnail_amd import _abi
_abi.lib_path = lambda: os.path.join(os.path.dirname(os.path.abspath(__file__)), "ablate_lib", "libraysnail_hip.so")
import torch; torch.cuda.set_device(0)
from raysnail_amd import scenes
cam, world, _, _ = scenes.rtow_13_1(800, 500)
photo = cam.take_photo().samples(64).depth(8).seed(1)
for _ in range(3):
    photo.shot(None, world); st = photo.last_stats
    print(f"ABLATED leaf: frame {st.ms:.2f} ms extend {st.kernel_ms:.2f} ms segs {st.segments}", flush=True)
