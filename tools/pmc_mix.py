# Per-kernel (per-dispatch mean) instruction mix, waits and VALU lane utilisation from
# tools/pmc_mix.sh passes.  usage: python tools/pmc_mix.py <outdir> [out.json]
import collections, csv, glob, json, os, sys


def short(name):
    return name.split("(")[0].replace("void ", "").replace("rs::", "").replace(" ", "")


def main():
    d = sys.argv[1]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(lambda: collections.defaultdict(set))
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k][r["Counter_Name"]].add(r["Dispatch_Id"])
    out = {}
    for k, c in acc.items():
        m = {n: v / max(1, len(disp[k][n])) for n, v in c.items()}
        g = lambda n: m.get(n, float("nan"))
        waves = g("SQ_WAVES")
        rec = dict(m)
        rec["dispatches"] = max(len(v) for v in disp[k].values())
        rec["valu_per_wave"] = g("SQ_INSTS_VALU") / waves
        rec["salu_per_wave"] = g("SQ_INSTS_SALU") / waves
        rec["vmem_rd_per_wave"] = g("SQ_INSTS_VMEM_RD") / waves
        rec["lds_per_wave"] = g("SQ_INSTS_LDS") / waves
        rec["branch_per_wave"] = g("SQ_INSTS_BRANCH") / waves
        rec["l2_hit"] = g("TCC_HIT_sum") / max(1e-9, g("TCC_HIT_sum") + g("TCC_MISS_sum"))
        rec["lane_util"] = g("SQ_THREAD_CYCLES_VALU") / (64.0 * g("SQ_ACTIVE_INST_VALU"))
        rec["wait_inst_frac"] = g("SQ_WAIT_INST_ANY") / g("SQ_WAVE_CYCLES")
        rec["wait_any_frac"] = g("SQ_WAIT_ANY") / g("SQ_WAVE_CYCLES")
        rec["valu_active_frac_of_wave_cycles"] = g("SQ_ACTIVE_INST_VALU") / g("SQ_WAVE_CYCLES")
        f64 = g("SQ_INSTS_VALU_ADD_F64") + g("SQ_INSTS_VALU_MUL_F64") + g("SQ_INSTS_VALU_FMA_F64") + g("SQ_INSTS_VALU_TRANS_F64")
        f32 = g("SQ_INSTS_VALU_FMA_F32") + g("SQ_INSTS_VALU_ADD_F32") + g("SQ_INSTS_VALU_MUL_F32")
        rec["f64_frac_of_valu"] = f64 / g("SQ_INSTS_VALU")
        rec["f32_frac_of_valu"] = f32 / g("SQ_INSTS_VALU")
        rec["int32_frac_of_valu"] = g("SQ_INSTS_VALU_INT32") / g("SQ_INSTS_VALU")
        out[k] = rec
    for k in sorted(out, key=lambda k: -out[k].get("SQ_WAVE_CYCLES", 0)):
        r = out[k]
        print(f"{k[:44]:44s} disp {r['dispatches']:3d} VALU/wave {r['valu_per_wave']:8.0f} SALU/wave {r['salu_per_wave']:6.0f} "
              f"VMEM/wave {r['vmem_rd_per_wave']:5.0f} LDS/wave {r['lds_per_wave']:5.0f} lane {r['lane_util']:.3f} "
              f"f64 {r['f64_frac_of_valu']:.2f} f32 {r['f32_frac_of_valu']:.2f} int {r['int32_frac_of_valu']:.2f} "
              f"waitinst {r['wait_inst_frac']:.2f} valuact {r['valu_active_frac_of_wave_cycles']:.2f}")
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
