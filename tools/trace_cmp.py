# dev: per-kernel durations of the last frame of each kernel trace given (frames end at k_accumulate)
# usage: python tools/trace_cmp.py <kernel_trace.csv> [...]
import csv, sys
for f in sys.argv[1:]:
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    acc = [i for i, r in enumerate(rows) if "accumulate" in r["Kernel_Name"] or "finalize" in r["Kernel_Name"]]
    a, b = acc[-3] if "finalize" in rows[acc[-1]]["Kernel_Name"] else acc[-2], acc[-1]
    ks = [k for k in rows[a + 1:b + 1] if "rocclr" not in k["Kernel_Name"]]
    dur = lambda k: (int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e3
    tag = lambda k: "E" if "extend" in k["Kernel_Name"] else "S" if "shade" in k["Kernel_Name"] else "A"
    ext = [dur(k) for k in ks if tag(k) == "E"]
    sh = [dur(k) for k in ks if tag(k) == "S"]
    print(f.split("/")[-2], f"busy {sum(map(dur, ks)):.0f} us  extend {sum(ext):.0f}  shade {sum(sh):.0f}")
    print("  E", " ".join(f"{x:.0f}" for x in ext))
    print("  S", " ".join(f"{x:.0f}" for x in sh))
