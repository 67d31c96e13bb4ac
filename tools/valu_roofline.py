# VALU-issue roofline per kernel: wave-instructions issued (PMC, tools/pmc_mix.sh passes of a one-lane
# run) weighted by their SIMD cycles on gfx950 -- a wave64 f32 / integer VALU op occupies a SIMD for
# 2 cycles, an f64 op for 4 (MI355X_MICROARCH.md: FP64 vector = half the FP32 rate) -- against the
# chip's SIMD cycles over the kernel's duration (rocprofv3 kernel trace of the same one-lane command):
# util = sum(cycles) / (1024 SIMDs x 2.4 GHz x duration). Lane utilisation alongside.
# usage: python tools/valu_roofline.py <pmc_mix dir> <kernel_trace.csv> [out.json]
import collections, csv, glob, json, os, sys

SIMDS, CLK = 256 * 4, 2.4e9


def short(name):
    return name.split("(")[0].replace("void ", "").replace("rs::", "").replace(" ", "")


def main():
    d, trace = sys.argv[1], sys.argv[2]
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            tot[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    dur = collections.defaultdict(float)
    ndisp = collections.Counter()
    for r in csv.DictReader(open(trace)):
        k = short(r["Kernel_Name"])
        dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        ndisp[k] += 1
    out = {}
    for k, c in tot.items():
        if k not in dur or "VALU" not in " ".join(c):
            continue
        valu = c.get("SQ_INSTS_VALU", 0.0)
        f64 = sum(c.get(n, 0.0) for n in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                            "SQ_INSTS_VALU_TRANS_F64"))
        # the PMC run and the trace run render the same frames; counters are totals over all dispatches
        cyc = 2.0 * (valu - f64) + 4.0 * f64
        util = cyc / (SIMDS * CLK * dur[k]) if dur[k] > 0 else float("nan")
        lane = c.get("SQ_THREAD_CYCLES_VALU", 0.0) / (64.0 * c.get("SQ_ACTIVE_INST_VALU", 1.0))
        out[k] = {"valu_wave_insts": valu, "f64_share": f64 / valu if valu else 0.0, "seconds": dur[k],
                  "dispatches": ndisp[k], "valu_issue_util": util, "lane_util": lane,
                  "lane_weighted_util": util * lane}
        print(f"{k[:40]:40s} VALU issue {util:.3f} of the SIMD cycles, lanes {lane:.3f} -> {util * lane:.3f} "
              f"(f64 {f64 / valu:.2f} of VALU, {dur[k] * 1e3:.2f} ms over {ndisp[k]} dispatches)")
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
