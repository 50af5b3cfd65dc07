"""Print one step's kernel timeline from a rocprofv3 kernel trace (start offset, duration, gap to
the previous kernel on any queue).  Usage: timeline.py run_kernel_trace.csv [step_index_from_end]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
idx = [i for i, r in enumerate(rows) if "bag_fwd" in r["Kernel_Name"]]
s, e = idx[-k - 1], idx[-k]
t0 = int(rows[s]["Start_Timestamp"])
last_end = None
busy = 0
for r in rows[s:e]:
    n = r["Kernel_Name"].replace("tt::(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*", "", n)[:70]
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (st - last_end) / 1e3 if last_end else 0.0
    print(f"{(st - t0) / 1e3:8.1f} {(en - st) / 1e3:7.1f} gap{gap:7.1f} q{r['Queue_Id']:>2}  {n}")
    last_end = max(last_end or 0, en)
print(f"step span {(int(rows[e]['Start_Timestamp']) - t0) / 1e3:.1f} us")
