# dev: GPU occupancy of a rocprofv3 kernel trace over its last `frames` frames (a frame ends with its k_accumulate):
# the union of kernel intervals (busy), the time with >= 2 kernels running (overlap), and the idle gaps.
# usage: python tools/trace_busy.py <kernel_trace.csv> [frames]
import csv, sys
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"])
              for r in csv.DictReader(open(sys.argv[1])))
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 10
acc = [i for i, r in enumerate(rows) if "k_accumulate" in r[2]]
if len(acc) > frames:
    t0 = rows[acc[-frames - 1]][1]
    rows = [r for r in rows if r[0] >= t0]
t_start, t_end = min(r[0] for r in rows), max(r[1] for r in rows)
ev = sorted([(s, 1) for s, _, _, _ in rows] + [(e, -1) for _, e, _, _ in rows])
busy = over = 0
depth, last = 0, ev[0][0]
gaps = []
for t, d in ev:
    if depth >= 1: busy += t - last
    if depth >= 2: over += t - last
    if depth == 0 and t > last: gaps.append(t - last)
    depth += d
    last = t
span = t_end - t_start
print(f"{len(rows)} kernels over {span / 1e3:.1f} us ({frames} frames: {span / 1e3 / frames:.1f} us each): busy {busy / span:.3f}, "
      f">= 2 kernels {over / span:.3f}, idle gaps {len(gaps)} totalling {sum(gaps) / 1e3:.1f} us (largest {max(gaps or [0]) / 1e3:.1f} us)")
qs = {}
for s, e, n, q in rows:
    qs.setdefault(q, [0, 0.0])
    qs[q][0] += 1
    qs[q][1] += (e - s) / 1e3
for q, (n, us) in sorted(qs.items()):
    print(f"  queue {q}: {n} kernels, {us:.1f} us")
