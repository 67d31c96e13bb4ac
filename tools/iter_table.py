# dev: per-iteration table of the bench frame from a one-lane dev run with RS_DUMP_ITERS=1 (tools/gpu.sh iters):
# the queue counts the library printed per iteration and the kernel trace's launch durations (the extend --
# 'ext rest' = all its records: the front-run / rest split of earlier rounds' dev builds is gone -- and the
# shading), averaged over the frames after the first; ps per path for each.
# usage: python tools/iter_table.py <iters.log> <kernel_trace.csv>
import csv, re, sys
from collections import defaultdict


def main():
    log, trace = sys.argv[1], sys.argv[2]
    pat = re.compile(r"iter lane (\d+) t +(\d+): carried +(\d+) \(front +(\d+) back +(\d+)\) camera +(\d+) shaded +(\d+) "
                     r"\[(\d+) (\d+) (\d+) (\d+) (\d+)\] ended +(\d+)")
    frames, cur = [], []
    for line in open(log):
        m = pat.search(line)
        if not m:
            continue
        v = [int(x) for x in m.groups()]
        if v[1] == 0 and cur:
            frames.append(cur)
            cur = []
        cur.append(v)
    if cur:
        frames.append(cur)
    rows = sorted(csv.DictReader(open(trace)), key=lambda r: int(r["Start_Timestamp"]))
    fl, f = [], []
    for r in rows:
        n = r["Kernel_Name"]
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if "k_wfs_extend" in n:
            f.append(("E", d))
        elif "k_wfs_shade_all" in n:
            f.append(("S", d))
        elif "k_accumulate" in n and f:
            fl.append(f)
            f = []
    per_it = defaultdict(lambda: defaultdict(list))
    for fr in fl[1:]:
        # an iteration: its extend launches, then its shading launches (one, or the split shading's two)
        its, prev = [], None
        for kind, d in fr:
            if kind == "E" and prev != "E":
                its.append(([], []))
            its[-1][0 if kind == "E" else 1].append(d)
            prev = kind
        for t, (es, ss) in enumerate(its):
            per_it[t]["E"].append(es)
            per_it[t]["S"].append(sum(ss))
    counts = frames[-1] if frames else []
    print(f"{'t':>2} {'front':>9} {'back':>9} {'camera':>9} {'shaded':>9} {'ended':>9} | {'ext front us':>12} {'ps/ray':>7} "
          f"{'ext rest us':>12} {'ps/ray':>7} {'shade us':>9} {'ps/path':>7}")
    tot = defaultdict(float)
    for t in sorted(per_it):
        es = per_it[t]["E"]
        k = len(es[0])
        ext = [sum(e[i] for e in es) / len(es) for i in range(k)]
        sh = sum(per_it[t]["S"]) / len(per_it[t]["S"])
        c = counts[t] if t < len(counts) else [0] * 13
        front, back, cam, shaded, ended = c[3], c[4], c[5], c[6], c[12]
        if k == 2:
            ef, er = ext
            rest = back + cam
        else:
            ef, er = 0.0, ext[0]
            rest = front + back + cam
        tot["ef"] += ef; tot["er"] += er; tot["sh"] += sh
        print(f"{t:>2} {front:>9} {back:>9} {cam:>9} {shaded:>9} {ended:>9} | {ef:>12.1f} {1e6 * ef / max(front, 1):>7.1f} "
              f"{er:>12.1f} {1e6 * er / max(rest, 1):>7.1f} {sh:>9.1f} {1e6 * sh / max(shaded, 1):>7.1f}")
    print(f"frame: extend front {tot['ef']:.1f} us, extend rest {tot['er']:.1f} us, shading {tot['sh']:.1f} us "
          f"({len(fl) - 1} frames averaged)")


if __name__ == "__main__":
    main()
