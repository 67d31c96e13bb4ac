# dev: for several library builds (tools/build_variant.sh), time the bench frame and its N=8 row share
# (rows 0::8) with asynchronous rs_render_device calls, and hash the full frame (bitwise check
# against the first, parity-tested build).  usage: python tools/variant_share.py [lib.so ...]
import glob, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, time, hashlib
sys.path.insert(0, ROOT)
from raysnail_amd import _abi
_abi.lib_path = lambda: LIB
import torch; torch.cuda.set_device(0)
from raysnail_amd import scenes
cam, world, _, _ = scenes.rtow_13_1(800, 500)
photo = cam.take_photo().samples(64).depth(8).seed(1)
ds = world.device_scene()
fr = torch.zeros((500, 800, 4), dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
def run(rs, n):
    st = photo.rows(0, 0, rs).settings()
    for _ in range(3): ds.render_device(cam.desc, st, fr.data_ptr(), s, stats=False)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(n): ds.render_device(cam.desc, st, fr.data_ptr(), s, stats=False)
    torch.cuda.synchronize(); return (time.perf_counter() - t) / n * 1e3
full = min(run(1, 10) for _ in range(2)); share = min(run(8, 20) for _ in range(2))
ds.render_device(cam.desc, photo.rows(0, 0, 1).settings(), fr.data_ptr(), s, stats=False); torch.cuda.synchronize()
md5 = hashlib.md5(fr.cpu().numpy().tobytes()).hexdigest()[:12]
print(f"full {full:.3f} ms share8 {share:.3f} ms eff {full / (8 * share):.3f} md5 {md5}")
'''


def main():
    libs = sys.argv[1:] or [os.path.join(ROOT, "raysnail_amd/lib/libraysnail_hip.so")] + sorted(
        glob.glob(os.path.join(ROOT, "raysnail_amd/lib/var_*.so")))
    for spec in libs:  # lib.so[:VAR=value,VAR=value] -- environment for that run (e.g. RS_LANES=1)
        lib, _, envs = spec.partition(":")
        env = dict(os.environ)
        for kv in filter(None, envs.split(",")):
            k, _, v = kv.partition("=")
            env[k] = v
        code = CHILD.replace("ROOT", repr(ROOT)).replace("LIB", repr(lib))
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
        out = r.stdout.strip().splitlines()
        print(f"{os.path.basename(lib)} {envs}: {out[-1] if out else 'FAILED rc=%d %s' % (r.returncode, r.stderr[-400:])}", flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
