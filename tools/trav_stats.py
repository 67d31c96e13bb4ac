# dev: traversal counters of the bench frame (and other scenes) from a -DRS_TRAV_STATS build
# (tools/build_variant.sh stats -DRS_TRAV_STATS), per ray category: camera rays (and the bounce-synchronous
# wavefront's rays), the carried front run (light-sample rays), the rest (BSDF / other rays).
# usage: python tools/trav_stats.py [lib.so] [scene,scene,...]
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from raysnail_amd import _abi
lib_file = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "raysnail_amd/lib/var_stats.so")
_abi.lib_path = lambda: lib_file
import torch; torch.cuda.set_device(0)
from raysnail_amd import scenes
lib = _abi.load()
out = (C.c_ulonglong * 128)()
# scene -> (builder, spp, depth, translation unit of its scene mode: rs_kernels.hip RS_TU)
CASES = {"rtow": (lambda: scenes.rtow_13_1(800, 500)[:2], 64, 8, 1),
         "mesh": (lambda: scenes.mesh_scene(960, 540), 16, 50, 2),
         "example": (lambda: scenes.example_sdl(800, 500), 16, 50, 3),
         "quadric": (lambda: scenes.quadric_sdl(512, 512), 16, 50, 4)}
CATS = ["camera/bsync", "front(light)", "rest(bsdf)"]
names = sys.argv[2].split(",") if len(sys.argv) > 2 else ["rtow"]
for name in names:
    build, spp, depth, tu = CASES[name]
    fn = getattr(lib, f"rs_debug_trav_stats_{tu}")
    cam, world = build()
    photo = cam.take_photo().samples(spp).depth(depth).seed(1)
    photo.shot(None, world)
    assert fn(out, 1) == 0, "reading the counters failed (a fault in the frame before?)"
    photo.shot(None, world)
    assert fn(out, 1) == 0, "reading the counters failed (a fault in the frame before?)"
    for c, cname in enumerate(CATS):
        v = out[32 * c:32 * c + 32]
        nodes, leaves, rays, wmax, lanes, waves, witer = v[:7]
        if not rays:
            continue
        print(f"{name} {cname:13s}: rays {rays} nodes/ray {nodes/max(rays,1):.2f} leaves/ray {leaves/max(rays,1):.2f} "
              f"wave-max nodes {wmax/max(waves,1):.2f} live lanes/wave {lanes/max(waves,1):.1f} "
              f"lane efficiency {(nodes/max(rays,1))/max(wmax/max(waves,1),1e-9):.3f} "
              # leaf passes exist only in the near-first walks (bvh4_step, the flat leaf FIFO); the nest modes'
              # deferred walk lists a ray's leaves and tests them in a loop of its own (no passes counted)
              + (f"leaf passes/wave {witer/max(waves,1):.2f} leaf-pass lane use {leaves/(64*witer):.3f}" if witer
                 else "leaf passes n/a (deferred leaf list)"), flush=True)
        hist = list(v[8:24])
        tot = max(1, sum(hist))
        print("   node steps per ray, 8-wide buckets (%):", " ".join(f"{8*b}:{100*h/tot:.1f}" for b, h in enumerate(hist)),
              flush=True)
