# dev: per-kernel summary of a rocprofv3 kernel trace: launches, total / average duration, VGPRs, AGPRs, scratch
# bytes per lane, LDS bytes per block.  usage: python tools/kernel_table.py <kernel_trace.csv> [name filter]
import csv, sys
from collections import OrderedDict
flt = sys.argv[2] if len(sys.argv) > 2 else ""
k = OrderedDict()
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if flt not in n:
        continue
    e = k.setdefault(n, {"n": 0, "us": 0.0, "vgpr": r["VGPR_Count"], "agpr": r.get("Accum_VGPR_Count", ""),
                         "scratch": r["Scratch_Size"], "lds": r["LDS_Block_Size"]})
    e["n"] += 1
    e["us"] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
for n, e in sorted(k.items(), key=lambda x: -x[1]["us"]):
    print(f"{e['us']:11.1f} us {e['n']:5d} x {e['us'] / e['n']:9.1f} us  vgpr {e['vgpr']:>3} agpr {e['agpr']:>2} "
          f"scratch {e['scratch']:>4} lds {e['lds']:>6}  {n[:110]}")
