"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs) into per-kernel HBM
bytes per launch, corrected as MI355X_MICROARCH.md §HBM prescribes for gfx950 (FETCH_SIZE reads
half the bytes of a wide stream: x2; kB -> bytes x1024).
usage: python tools/collect_pmc.py <fetch_csv> <write_csv> <out_json> [profile_tag]"""
import csv
import json
import sys


def kernel_key(name):
    return name.split("(")[0].replace("void ", "").split("<")[0].replace("rs::", "")


def main(fetch_csv, write_csv, out_json, tag=None):
    acc = {}
    for ctr, f in (("FETCH_SIZE", fetch_csv), ("WRITE_SIZE", write_csv)):
        for r in csv.DictReader(open(f)):
            k = kernel_key(r["Kernel_Name"])
            if not k.startswith("k_"):
                continue
            acc.setdefault(k, {"FETCH_SIZE": [], "WRITE_SIZE": []})[ctr].append(float(r["Counter_Value"]))
    out = {}
    for k, d in acc.items():
        if not d["FETCH_SIZE"] or not d["WRITE_SIZE"]:
            continue
        f = sum(d["FETCH_SIZE"]) / len(d["FETCH_SIZE"])
        w = sum(d["WRITE_SIZE"]) / len(d["WRITE_SIZE"])
        out[k] = {"FETCH_SIZE_kB": f, "WRITE_SIZE_kB": w, "launches_sampled": len(d["FETCH_SIZE"]),
                  "hbm_bytes_per_launch": (2.0 * f + w) * 1024.0,
                  "note": "gfx950: FETCH_SIZE x2, kB x1024 (MI355X_MICROARCH.md HBM)"}
    if tag:
        out["_round"] = tag   # bench.py reports it next to the traffic figure
    json.dump(out, open(out_json, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:5])
