# dev: time the bench frame with several library builds (tools/build_variant.sh) in turn; frames are
# hashed so every variant can be checked bitwise against the first (the in-tree, parity-tested lib).
# usage: python tools/variant_bench.py [--scene=key] [lib.so[:VAR=value,VAR=value] ...]
#        (default: all raysnail_amd/lib/var_*.so; the VAR=value pairs are that run's environment)
import glob, hashlib, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import os, sys, hashlib
sys.path.insert(0, ROOT)
from raysnail_amd import _abi
_abi.lib_path = lambda: LIB
import torch; torch.cuda.set_device(0)
from raysnail_amd import scenes
cam, world = SCENE
photo = cam.take_photo().samples(SPP).depth(DEPTH).seed(1)
best = None
for _ in range(4):
    img = photo.shot(None, world); st = photo.last_stats
    if best is None or st.ms < best[0]: best = (st.ms, st.kernel_ms)
print(f"frame {best[0]:.2f} ms extend {best[1]:.2f} ms {st.samples/best[0]/1e3:.1f} Msamples/s segs {st.segments} md5 {hashlib.md5(img.tobytes()).hexdigest()[:12]}")
'''
SCENES = {"rtow": ("scenes.rtow_13_1(800, 500)[:2]", 64, 8),
          "example": ("scenes.example_sdl(800, 500)", 64, 8),
          "quadric": ("scenes.quadric_sdl(512, 512)", 16, 8),
          "mesh": ("scenes.mesh_scene(480, 270, 64, 120)", 16, 8),
          "c4": ("scenes.quadric_sdl(512, 512)", 64, 50),
          "c5": ("scenes.mesh_scene(960, 540)", 16, 50),
          "x1": ("scenes.all_feature_scene(400, 400)", 16, 50),
          "x2": ("scenes.cornell_smoke(300, 300)", 64, 50)}


def main():
    args = sys.argv[1:]
    scene = "rtow"
    if args and args[0].startswith("--scene="):
        scene = args.pop(0).split("=", 1)[1]
    libs = args or [os.path.join(ROOT, "raysnail_amd/lib/libraysnail_hip.so")] + sorted(
        glob.glob(os.path.join(ROOT, "raysnail_amd/lib/var_*.so")))
    expr, spp, depth = SCENES[scene]
    for spec in libs:
        lib, _, envs = spec.partition(":")
        env = dict(os.environ)
        for kv in filter(None, envs.split(",")):
            k, v = kv.split("=", 1)
            env[k] = v
        code = (CHILD.replace("ROOT", repr(ROOT)).replace("LIB", repr(lib)).replace("SCENE", expr)
                .replace("SPP", str(spp)).replace("DEPTH", str(depth)))
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
        out = r.stdout.strip().splitlines()
        print(f"{scene} {os.path.basename(lib)}{':' + envs if envs else ''}: {out[-1] if out else 'FAILED rc=%d %s' % (r.returncode, r.stderr[-400:])}",
              flush=True)
        if r.returncode != 0:
            sys.exit(r.returncode)


if __name__ == "__main__":
    main()
