# dev: the kernel timeline of the last `n` kernels of a rocprofv3 kernel trace (start / end offsets
# in us from the first, duration, grid, queue). usage: timeline.py <kernel_trace.csv> [n]
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
sel = rows[-n:]
t0 = int(sel[0]["Start_Timestamp"])
busy = 0.0
end_max = 0
for r in sel:
    s = (int(r["Start_Timestamp"]) - t0) / 1e3
    e = (int(r["End_Timestamp"]) - t0) / 1e3
    print(f"{s:9.1f} {e:9.1f} {e - s:8.1f} q{r['Queue_Id']:>2} {int(r['Grid_Size_X']) // 256:>8} {r['Kernel_Name'][:64]}")
