"""Fold a tools/profile_round.sh output directory into committed summaries under profiles/:
<tag>_kernel_stats.csv (rocprofv3 --stats as produced), <tag>_summary.md (per-kernel time and
PMC HBM traffic per launch) and <tag>_pmc_traffic.json (per-op HBM bytes per launch, read by
bench.py for roofline.traffic).

PMC corrections (MI355X_MICROARCH.md, 'HBM / rocprofv3'): FETCH_SIZE and WRITE_SIZE are reported
in KiB; on gfx950 FETCH_SIZE counts half of the bytes of wide (16 B/lane) coalesced reads, so it is
doubled; WRITE_SIZE is exact for 16 B/lane stores.  Infinity-Cache hits are included in both, so the
figures are L2<->fabric bytes, an upper bound on HBM bytes."""
import csv
import glob
import json
import os
import re
import shutil
import sys
from collections import defaultdict

# kernel-name pattern -> the C-ABI op (bench.py 'abi') it belongs to
OPS = [
    (r"bag_fwd", "tt_bag_mean_fwd"),
    (r"bag_plan_keys|bag_plan_bounds|bag_plan_starts|bag_plan_pieces|plan_sort_|bag_bwd_mark|bag_piece_count"
     r"|bag_piece_list|radix_sort|onesweep|rocprim", "tt_bag_plan"),
    (r"bag_scale_rows|bag_piece_sum|bag_bwd_reduce_kernel<.*true>|bag_bwd_reduce_generic_kernel<true>"
     r"|bag_bwd_reduce_sliced_kernel<\d+, \d+, true", "tt_bag_mean_bwd_adamw_planned"),
    (r"bag_bwd_reduce", "tt_bag_mean_bwd_planned"),
    (r"score_bf16_kernel<0|score_f32_kernel<0|score_split_fwd|prep_rows|prep_qd|shift_kernel|fwd_combine", "tt_inbatch_fwd"),
    (r"score_bf16_kernel<1|score_f32_kernel<1|score_ddp_kernel|score_split_ddp|to_log2|bwd_combine", "tt_inbatch_bwd"),
    (r"adamw_(vec4|scalar)", "tt_adamw"),
    (r"adamw_multi_ex", "tt_adamw_multi_ex"),
    (r"adamw_multi|adam_prepare", "tt_adamw_multi"),
    (r"multi_neg_fwd", "tt_multi_neg_fwd"),
    (r"multi_neg_bwd", "tt_multi_neg_bwd"),
    (r"triplet_fwd", "tt_triplet_fwd"),
    (r"triplet_bwd", "tt_triplet_bwd"),
    (r"l2norm_fwd", "tt_l2norm_fwd"),
    (r"l2norm_bwd", "tt_l2norm_bwd"),
    (r"colsum", "tt_colsum"),
    (r"relu_bwd", "tt_relu_bwd"),
    (r"head_gemm|head_normalize", "tt_head_gemm"),
    (r"head_wgrad", "tt_head_wgrad"),
    (r"l2_prep_kernel|l2_prep128_kernel", "tt_inbatch_l2_prep"),
    (r"split_planes", "tt_head_split_ff"),
    (r"Cijk_", "hipBLASLt GEMM (tower FF)"),
]


def short(name: str) -> str:
    if name.startswith("Cijk"):
        return name[:60]
    name = name.replace("tt::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    name = name.replace("void ", "").replace("rocprim::ROCPRIM_400200_NS::detail::", "rocprim::")
    return re.sub(r"\((?!\)).*$", "", name)[:110] if not name.startswith("_Z") else name[:80]


def op_of(name: str) -> str:
    for pat, op in OPS:
        if re.search(pat, name):
            return op
    return "other (torch/runtime)"


MARKER = "stamp_kernel"  # bench.py brackets its timed steps with two tt_stamp launches (window_marker)


def _window(rows, key):
    """(lo, hi) of `key` between the first two marker dispatches (bench.py's timed region comes before
    any stamped per-op timing), or None without markers."""
    marks = sorted(key(r) for r in rows if MARKER in r["Kernel_Name"])
    return (marks[0], marks[1]) if len(marks) >= 2 else None


def trace_stats(path: str):
    """Per-kernel (calls, total ns) from the kernel trace, restricted to the timed steps when bench
    left its window markers; None if the trace has no markers (then the --stats summary is used)."""
    files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        return None
    with open(files[0]) as fh:
        rows = list(csv.DictReader(fh))
    win = _window(rows, lambda r: int(r["Start_Timestamp"]))
    if win is None:
        return None
    out = defaultdict(lambda: [0, 0])
    for r in rows:
        t = int(r["Start_Timestamp"])
        if win[0] < t < win[1] and MARKER not in r["Kernel_Name"]:
            out[r["Kernel_Name"]][0] += 1
            out[r["Kernel_Name"]][1] += int(r["End_Timestamp"]) - t
    return out


def pmc(path: str, counter: str):
    rows = []
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += [r for r in csv.DictReader(fh) if r.get("Counter_Name") == counter]
    win = _window(rows, lambda r: int(r["Dispatch_Id"]))
    if win is not None:  # the dispatches of the timed steps only
        rows = [r for r in rows if win[0] < int(r["Dispatch_Id"]) < win[1] and MARKER not in r["Kernel_Name"]]
    return [(r["Kernel_Name"], float(r["Counter_Value"])) for r in rows]


def main(outdir: str, tag: str):
    os.makedirs("profiles", exist_ok=True)
    stats = glob.glob(os.path.join(outdir, "ktrace", "**", "*kernel_stats.csv"), recursive=True)[0]
    shutil.copy(stats, f"profiles/{tag}_kernel_stats.csv")
    ts = trace_stats(os.path.join(outdir, "ktrace"))
    if ts is not None:  # the timed steps alone: bench set-up and the warmup steps left out
        ks = [{"Name": n, "Calls": c, "TotalDurationNs": t, "AverageNs": t / c} for n, (c, t) in ts.items()]
        scope = "the timed steps only (between bench.py's two window markers; set-up and warmup excluded)"
    else:
        with open(stats) as fh:
            ks = list(csv.DictReader(fh))
        scope = "the whole run (incl. warmup and set-up; no window markers in the trace)"
    # steps profiled = calls of the bag forward kernel (one launch per step); a trace without it
    # (a tools/mb.py run, tools/profile_mb.sh) is reported per launch, "calls/step" = calls
    steps = max((int(r["Calls"]) for r in ks if "bag_fwd" in r["Name"]), default=1)
    fetch = defaultdict(list)
    write = defaultdict(list)
    for n, v in pmc(os.path.join(outdir, "fetch"), "FETCH_SIZE"):
        fetch[n].append(v * 1024 * 2)
    for n, v in pmc(os.path.join(outdir, "write"), "WRITE_SIZE"):
        write[n].append(v * 1024)
    lines = [f"# Profile {tag}", "", "Source: `tools/profile_round.sh` over `bench.py`, or `tools/profile_mb.sh` over `tools/mb.py` when "
             "no bag kernel is in the trace (rocprofv3 --kernel-trace --stats; separate --pmc FETCH_SIZE and "
             "--pmc WRITE_SIZE passes).", "",
             f"Steps covered: {steps}, {scope}", "",
             "| kernel | op | calls/step | avg us | us/step | fetch MB/launch | write MB/launch |",
             "|---|---|---|---|---|---|---|"]
    per_op = defaultdict(lambda: {"us_per_step": 0.0, "fetch": 0.0, "write": 0.0})
    for r in sorted(ks, key=lambda r: -float(r["TotalDurationNs"])):
        n = r["Name"]
        calls = int(r["Calls"]) / steps
        avg = float(r["AverageNs"]) / 1e3
        f = sum(fetch[n]) / len(fetch[n]) if fetch.get(n) else None
        w = sum(write[n]) / len(write[n]) if write.get(n) else None
        op = op_of(n)
        per_op[op]["us_per_step"] += avg * calls
        per_op[op]["fetch"] += (f or 0.0) * calls
        per_op[op]["write"] += (w or 0.0) * calls
        lines.append(f"| `{short(n)}` | {op} | {calls:.2f} | {avg:.1f} | {avg * calls:.1f} | "
                     f"{'-' if f is None else f'{f / 1e6:.1f}'} | {'-' if w is None else f'{w / 1e6:.1f}'} |")
    lines += ["", "## Per op (summed over its kernels, per step)", "", "| op | us/step | fetch MB | write MB |",
              "|---|---|---|---|"]
    for op, d in sorted(per_op.items(), key=lambda kv: -kv[1]["us_per_step"]):
        lines.append(f"| {op} | {d['us_per_step']:.1f} | {d['fetch'] / 1e6:.1f} | {d['write'] / 1e6:.1f} |")
    open(f"profiles/{tag}_summary.md", "w").write("\n".join(lines) + "\n")
    traffic = {op: {"hbm_bytes_per_call": d["fetch"] + d["write"], "fetch_bytes": d["fetch"], "write_bytes": d["write"],
                    "device_us_per_step": d["us_per_step"]} for op, d in per_op.items()}
    json.dump({"tag": tag, "scope": scope, "note": "PMC FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, "
               "KiB->bytes; per step = per call for ops launched once per step", "ops": traffic},
              open(f"profiles/{tag}_pmc_traffic.json", "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
