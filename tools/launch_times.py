# dev: per-launch durations (us) of the extend / shade kernels in a rocprofv3 kernel trace
# usage: python tools/launch_times.py <kernel_trace.csv> [launches] [first]
#   default: the last 50 launches of each; with `first`, the first N
import csv, sys
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(sys.argv[1])))
per = int(sys.argv[2]) if len(sys.argv) > 2 else 50
first = len(sys.argv) > 3 and sys.argv[3] == "first"
for key in ("extend", "shade"):
    d = [(e - s) / 1e3 for s, e, n in rows if key in n]
    d = d[:per] if first else d[-per:]
    print(f"{key:7s} sum {sum(d):8.1f} us: " + " ".join(f"{x:.0f}" for x in d))
