"""Recompute bench.py's roofline field from a rocprofv3 kernel trace of the same bench.py run.

usage: python tools/trace_roofline.py <kernel_trace.csv> <bench line .json>

bench.py runs, in this order: `warmup` frames, `steps` timed (pipelined) frames, min(steps, 5) latency frames,
then `steps` statistics frames on one lane, each frame alone -- the frames its `avg_launch_ms` is event-timed on.
Every frame of the workload enqueues the same launches, so the statistics frames' extend launches are the
`launches_per_step` x `steps` dominant-kernel dispatches that follow the first (warmup + steps + latency) frames'
ones in dispatch order. Their mean duration gives `achieved` = alg_bytes_per_launch / mean and `frac`, which must
agree with the line's within the events' resolution (a few per cent).
"""
import csv
import json
import sys


def main():
    trace, line = sys.argv[1], sys.argv[2]
    d = json.loads(open(line).read().strip().splitlines()[-1])
    roof = d["roofline"]
    kname = roof["kernel"]
    lps = int(roof["launches_per_step"])
    steps, warm = int(d["steps"]), int(d["warmup"])
    before = warm + steps + min(steps, 5)
    rows = []
    with open(trace) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            # rs::k_wfs_extend<...> (camera part, carried part); not k_wfs_finish
            base = name.split("<")[0].split("::")[-1]
            if base == kname:
                rows.append((int(r["Dispatch_Id"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    sel = rows[before * lps:(before + steps) * lps]
    if len(sel) != steps * lps:
        sys.exit(f"trace holds {len(rows)} {kname} dispatches, expected at least {(before + steps) * lps}")
    mean_ns = sum(e - s for _, s, e in sel) / len(sel)
    alg = float(roof["alg_bytes_per_launch"])
    achieved = alg / (mean_ns * 1e-9) / 1e9
    frac = achieved / float(roof["peak"])
    out = {"kernel": kname, "dispatches_in_trace": len(rows), "statistics_frame_dispatches": len(sel),
           "first_dispatch_id": sel[0][0], "trace_mean_launch_ms": round(mean_ns / 1e6, 4),
           "line_avg_launch_ms": roof["avg_launch_ms"], "trace_achieved_GBs": round(achieved, 2),
           "line_achieved_GBs": roof["achieved"], "trace_frac": round(frac, 5), "line_frac": roof["frac"],
           "frac_rel_diff": round(frac / float(roof["frac"]) - 1.0, 4),
           "all_dispatches_mean_ms": round(sum(e - s for _, s, e in rows) / len(rows) / 1e6, 4)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
