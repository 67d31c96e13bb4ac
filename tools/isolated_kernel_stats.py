# Average duration of a kernel's dispatches that ran ALONE on the GPU (no other dispatch overlapping
# in time), from a rocprofv3 --kernel-trace CSV: what bench.py's event-timed roofline launches are
# (its stats frames run one wavefront lane). usage: isolated_kernel_stats.py <kernel_trace.csv> [prefix]
import csv, json, sys

rows = list(csv.DictReader(open(sys.argv[1])))
prefix = sys.argv[2] if len(sys.argv) > 2 else "k_wfs_extend"
d = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
            r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rs::", "")) for r in rows)
iso, all_ = [], []
for i, (s, e, n) in enumerate(d):
    if not n.startswith(prefix):
        continue
    all_.append(e - s)
    alone = all(not (s2 < e and s < e2) for j, (s2, e2, _) in enumerate(d[max(0, i - 64):i + 64], max(0, i - 64)) if j != i)
    if alone:
        iso.append(e - s)
out = {"kernel": prefix, "dispatches": len(all_), "isolated_dispatches": len(iso),
       "avg_ms_all": round(sum(all_) / max(1, len(all_)) / 1e6, 4),
       "avg_ms_isolated": round(sum(iso) / max(1, len(iso)) / 1e6, 4)}
print(json.dumps(out))
