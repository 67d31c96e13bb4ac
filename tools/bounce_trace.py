# dev: per-bounce kernel durations of one scene (run under `rocprofv3 --kernel-trace`, then
# `python tools/bounce_trace.py --report <kernel_trace.csv> [depth]`)
# usage: python tools/bounce_trace.py <scene-key> [lanes]   (scene keys of tools/variant_bench.py)
import csv, os, sys
from collections import defaultdict
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def report(path, depth):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    by = defaultdict(list)
    for r in rows:
        by[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for name, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        print(f"{name[:60]:60s} n={len(d):5d} total {sum(d)/1e3:8.2f} ms")
    for name, d in by.items():
        if "extend" not in name and "shade" not in name:
            continue
        if len(d) % depth:
            continue
        frames = len(d) // depth
        per = [sum(d[f * depth + b] for f in range(1, frames)) / max(1, frames - 1) for b in range(depth)]
        print(name[:60], "per bounce (us, frames 2..):", " ".join(f"{x:.0f}" for x in per))


if __name__ == "__main__":
    if sys.argv[1] == "--report":
        report(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 50)
        sys.exit(0)
    os.environ["RS_LANES"] = sys.argv[2] if len(sys.argv) > 2 else "1"
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from variant_bench import SCENES
    import torch
    torch.cuda.set_device(0)
    from raysnail_amd import scenes  # noqa: F401
    expr, spp, depth = SCENES[sys.argv[1]]
    cam, world = eval(expr)
    photo = cam.take_photo().samples(spp).depth(depth).seed(1)
    for _ in range(3):
        photo.shot(None, world)
        st = photo.last_stats
        print(f"{st.ms:.2f} ms kernel {st.kernel_ms:.2f} ms segs {st.segments}", flush=True)
