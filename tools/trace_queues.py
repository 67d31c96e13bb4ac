# dev: per hardware queue / stream of a rocprofv3 kernel trace (its second half): kernels, busy time, gaps between
# consecutive kernels on the queue; then the first 60 kernels of that half in start order.
# usage: python tools/trace_queues.py <kernel_trace.csv>
import csv, sys, collections
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-40:], r["Queue_Id"], r.get("Stream_Id",""))
              for r in csv.DictReader(open(sys.argv[1])))
rows = rows[len(rows)//2:]  # steady state
byq = collections.defaultdict(list)
for r in rows: byq[(r[3], r[4])].append(r)
for q, rs in sorted(byq.items()):
    gaps = [b[0]-a[1] for a, b in zip(rs, rs[1:])]
    dur = sum(r[1]-r[0] for r in rs)
    gaps.sort()
    print("queue/stream", q, "kernels", len(rs), "busy us %.1f" % (dur/1e3), "gap median us %.1f" % (gaps[len(gaps)//2]/1e3 if gaps else 0),
          "gap p90 %.1f" % (gaps[int(len(gaps)*0.9)]/1e3 if gaps else 0))
t0, t1 = rows[0][0], rows[-1][1]
print("span ms %.3f kernels %d" % ((t1-t0)/1e6, len(rows)))
for r in rows[:60]:
    print("%9.1f %7.1f %s q%s s%s" % ((r[0]-t0)/1e3, (r[1]-r[0])/1e3, r[2], r[3], r[4]))
