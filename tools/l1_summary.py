# dev: L1 (TCP) / L2 (TCC) counters per kernel from a rocprofv3 --pmc counter_collection.csv (tools/gpu.sh l1):
# tag accesses, L1 -> L2 read requests per access, mean L2 read latency, L2 hit rate.
# usage: python tools/l1_summary.py <counter_collection.csv>
import csv, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].replace("void ", "").split("(")[0]
    acc[n][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[n].add(r["Dispatch_Id"])
print("L1 (TCP) / L2 (TCC) counters (rocprofv3 --pmc, one pass)")
for n, c in acc.items():
    a = c.get("TCP_TOTAL_CACHE_ACCESSES_sum", 0.0)
    rq = c.get("TCP_TCC_READ_REQ_sum", 0.0)
    lat = c.get("TCP_TCC_READ_REQ_LATENCY_sum", 0.0)
    h, m = c.get("TCC_HIT_sum", 0.0), c.get("TCC_MISS_sum", 0.0)
    if a == 0:
        continue
    print(f"{n[:45]:45s} dispatches {len(disp[n]):3d}  L1 tag accesses {a:9.3g}  L1->L2 read reqs {rq:9.3g} "
          f"({rq / a:.3f} per access)  mean L2 read latency {lat / max(rq, 1):5.0f} cycles  L2 hit {h / max(h + m, 1):.3f}")
