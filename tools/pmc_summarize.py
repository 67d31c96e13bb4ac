# summarise tools/pmc_scene.sh output: per-launch means of each counter for kernels matching a substring
import csv, glob, os, sys, collections
d, pat = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(float)
launches = collections.defaultdict(set)
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if pat not in r["Kernel_Name"]:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        launches[r["Counter_Name"]].add(r["Dispatch_Id"])
out = {k: v / max(1, len(launches[k])) for k, v in acc.items()}
for k in sorted(out):
    print(f"{k:32s} {out[k]:.4g}")
g = lambda k: out.get(k, float("nan"))
print("--")
print("VALU lane util (THREAD_CYCLES_VALU / 64 ACTIVE_INST_VALU):", g("SQ_THREAD_CYCLES_VALU") / (64 * g("SQ_ACTIVE_INST_VALU")))
print("VALU busy per SIMD (ACTIVE_INST_VALU*4 / (GRBM_GUI_ACTIVE * 1024 SIMDs)):", 4 * g("SQ_ACTIVE_INST_VALU") / (g("GRBM_GUI_ACTIVE") * 1024))
print("L2 hit rate:", g("TCC_HIT_sum") / (g("TCC_HIT_sum") + g("TCC_MISS_sum")))
print("VALU insts per wave:", g("SQ_INSTS_VALU") / g("SQ_WAVES"), " VMEM_RD per wave:", g("SQ_INSTS_VMEM_RD") / g("SQ_WAVES"))
print("wait fraction (WAIT_INST_ANY / WAVE_CYCLES):", g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES"))
