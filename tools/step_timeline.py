"""Print one graph-replayed step's kernel sequence (start offset, duration, queue, gap on the
critical queue) from a rocprofv3 --kernel-trace CSV.  Usage: step_timeline.py run_kernel_trace.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "bag_fwd_kernel" in r["Kernel_Name"]]
k = len(idx) // 2
a, b = idx[k], idx[k + 1]
t0 = int(rows[a]["Start_Timestamp"])
busy = {}
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r["Queue_Id"]
    busy[q] = busy.get(q, 0) + (e - s)
    print("%8.1f %7.1f q%s %s" % ((s - t0) / 1e3, (e - s) / 1e3, q, r["Kernel_Name"][:90]))
print("step %.1f us; busy per queue (us): %s" % ((int(rows[b]["Start_Timestamp"]) - t0) / 1e3,
                                                {q: round(v / 1e3, 1) for q, v in busy.items()}))
