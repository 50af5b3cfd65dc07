"""Summarise tools/ab_bench.sh runs: per variant the ms/step of every round, median, and the
eager per-op times (ms) of the scorer and table-update ops."""
import glob
import json
import os
import statistics
import sys

d = sys.argv[1]
res = {}
for f in sorted(glob.glob(os.path.join(d, "*_*.log"))):
    name = os.path.basename(f).rsplit("_", 1)[0]
    try:
        line = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f"{f}: no JSON line ({e})")
        continue
    r = res.setdefault(name, {"ms": [], "ops": {}})
    r["ms"].append(line["ms_per_step"])
    for k in line.get("kernels", []):
        r["ops"].setdefault(k["abi"], []).append(k["mean_ms"])
        for p, v in (k.get("pass_ms") or {}).items():
            r["ops"].setdefault(k["abi"] + ":" + p, []).append(v)
for name, r in res.items():
    print(f"{name:>16}: ms/step {' '.join(f'{x:.4f}' for x in r['ms'])}  median {statistics.median(r['ms']):.4f}")
    for op, v in sorted(r["ops"].items()):
        print(f"{'':>18}{op:<44} {statistics.median(v):.4f}")
