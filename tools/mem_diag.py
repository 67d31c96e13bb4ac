# dev: device memory held across scenes in one process: free memory before, after a C3-shaped frame on 3 slots, and
# after the scene is dropped (the pools must be given back).  usage: python tools/mem_diag.py
import gc, os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch; torch.cuda.set_device(0)
from raysnail_amd import scenes
from oracle.binding import OracleScene
GB = 1 << 30
out = {"free0": torch.cuda.mem_get_info()[0] / GB}
cam, world = scenes.rtow_13_1(1920, 1080)[:2]
ds = world.device_scene()
photo = cam.take_photo().samples(256).depth(50).seed(1)
frame = torch.zeros((1080, 1920, 4), dtype=torch.float32, device="cuda")
for _ in range(3):
    ds.render_device(cam.desc, photo.settings(), frame.data_ptr(), torch.cuda.current_stream().cuda_stream, stats=False)
torch.cuda.synchronize()
out["free_after_3_slots"] = torch.cuda.mem_get_info()[0] / GB
orc = OracleScene(world)
del ds, frame
world = None
out["free_after_del_world_oracle_alive"] = torch.cuda.mem_get_info()[0] / GB
del orc
gc.collect()
torch.cuda.empty_cache()
out["free_after_all"] = torch.cuda.mem_get_info()[0] / GB
print(json.dumps({k: round(v, 2) for k, v in out.items()}), flush=True)
