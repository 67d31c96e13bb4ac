# dev: summary of interleaved bench.py A/B runs (tools/gpu.sh ab / variants): median ms/frame and Msamples/s per side.
# usage: python tools/ab_report.py base1.json base2.json ... -- new1.json new2.json ...
#        python tools/ab_report.py <name>_<rep>.json ...     (grouped by <name>)
import json, os, re, statistics, sys
from collections import defaultdict


def load(paths):
    return [json.loads(open(p).read().strip().splitlines()[-1]) for p in paths]


def line(name, runs):
    ms = [d["ms_per_step"] for d in runs]
    ext = [d["roofline"]["avg_launch_ms"] for d in runs]
    sh = [d.get("row_share", {}).get("ms_per_share", 0.0) for d in runs]
    print(f"{name:14s} ms/frame {' '.join(f'{x:.3f}' for x in ms)}  median {statistics.median(ms):.3f}  "
          f"Msamples/s {statistics.median([d['value'] for d in runs]):.1f}  extend {statistics.median(ext):.4f} ms/launch  "
          f"share {statistics.median(sh):.4f} ms")


def main():
    a = sys.argv[1:]
    if "--" in a:
        k = a.index("--")
        line("base", load(a[:k]))
        line("new", load(a[k + 1:]))
        return
    groups = defaultdict(list)
    for p in a:
        groups[re.sub(r"_\d+\.json$", "", os.path.basename(p))].append(p)
    for name in sorted(groups):
        line(name, load(sorted(groups[name])))


if __name__ == "__main__":
    main()
