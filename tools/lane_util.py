# dev: VALU lane utilisation per kernel from a rocprofv3 --pmc pass with SQ_THREAD_CYCLES_VALU and
# SQ_ACTIVE_INST_VALU (tools/lane_util.sh): util = THREAD_CYCLES_VALU / (64 * ACTIVE_INST_VALU), the
# fraction of a wave's 64 lanes that execute its VALU instructions (1.0 = no divergence).
# usage: python tools/lane_util.py <counter_collection.csv> [out.json]
import csv, json, sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "").replace("rs::", "")


def main():
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(sys.argv[1])):
        k = short(r["Kernel_Name"])
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    out = {}
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_ACTIVE_INST_VALU", 0)):
        a = c.get("SQ_ACTIVE_INST_VALU", 0.0)
        if a <= 0:
            continue
        out[k] = {"dispatches": len(disp[k]), "lane_util": c.get("SQ_THREAD_CYCLES_VALU", 0.0) / (64.0 * a),
                  **{n: v for n, v in c.items()}}
        print(f"{k:40s} dispatches {len(disp[k]):4d} lane_util {out[k]['lane_util']:.3f}")
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
