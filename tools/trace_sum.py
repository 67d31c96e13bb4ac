# dev: per-kernel totals of the second half of a rocprofv3 kernel trace (passes_trace.py renders everything twice)
# divided by K frames.  usage: python tools/trace_sum.py <kernel_trace.csv> K
import csv, sys
from collections import OrderedDict
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(sys.argv[1])))
K = int(sys.argv[2])
rows = [r for r in rows if "rs::" in r[2]]
half = rows[len(rows) // 2:]
k = OrderedDict()
for s, e, n in half:
    n = n.split("(")[0].replace("rs::", "")
    d = k.setdefault(n, [0, 0.0])
    d[0] += 1
    d[1] += (e - s) / 1e3
tot = sum(v[1] for v in k.values())
span = (half[-1][1] - half[0][0]) / 1e3
print(f"launches {len(half)}  kernel us per frame {tot / K:.1f}  span us per frame {span / K:.1f}")
for n, (c, us) in sorted(k.items(), key=lambda x: -x[1][1]):
    print(f"{us / K:9.1f} us/frame {c:5d} launches  {us / c:8.1f} us avg  {n}")
