"""Summarise tools/pmc_scorer.sh output: per scorer kernel, average duration and counter values.
Usage: pmc_report.py OUTDIR [JSON]: with JSON, also write the per-pass MFMA utilisation and the
engines' average durations there (bench.py reports them beside the scorer's algorithmic rate).
pmc_report.py OUTDIR --match SUBSTR: group the counters per kernel name containing SUBSTR instead
(tools/pmc_kernels.sh output)."""
import csv, glob, json, sys, collections, re
out = sys.argv[1]
MATCH = sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--match" else None
if MATCH:
    sys.argv = sys.argv[:2]


def _pass(name: str) -> str:
    if MATCH:
        return re.sub(r"\(.*", "", name.replace("tt::(anonymous namespace)::", "").replace("void ", ""))[:70]
    """forward engines: score_bf16_kernel<0, ...> (Li0E), score_ws_kernel, score_split_fwd_kernel"""
    return "fwd" if ("<0," in name or "Li0E" in name or "score_ws" in name or "split_fwd" in name) else "bwd"

js = {"passes": {}}
ks = list(csv.DictReader(open(glob.glob(f"{out}/ks/**/*kernel_stats.csv", recursive=True)[0])))
for r in ks:
    n = re.sub(r"\(.*", "", r["Name"].replace("tt::(anonymous namespace)::", "").replace("void ", ""))[:60]
    print(f"{n:62s} calls {r['Calls']:>4s} avg {float(r['AverageNs'])/1e3:8.1f} us")
    if n.startswith("score_"):
        js["passes"].setdefault(_pass(n), {})["engine_us"] = round(
            float(r["AverageNs"]) / 1e3, 2)
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if (MATCH or "score_") in r["Kernel_Name"]:
            k = _pass(r["Kernel_Name"])
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    a = {c: sum(v) / len(v) for c, v in d.items()}
    print(k, {c: f"{v:.3g}" for c, v in sorted(a.items())})
    if "SQ_VALU_MFMA_BUSY_CYCLES" in a and "GRBM_GUI_ACTIVE" in a:
        # MFMA busy cycles summed over SIMDs vs (GUI_ACTIVE/8 XCDs) x 1024 SIMDs
        u = a['SQ_VALU_MFMA_BUSY_CYCLES'] / (a['GRBM_GUI_ACTIVE'] / 8 * 1024)
        print(f"  MFMA util {u:.3f}")
        js["passes"].setdefault(k, {})["mfma_busy"] = round(u, 4)
    if "SQ_LDS_BANK_CONFLICT" in a:
        print(f"  LDS conflict frac {a['SQ_LDS_BANK_CONFLICT'] / max(a['SQ_LDS_IDX_ACTIVE'], 1):.3f}")
    if "SQ_WAVE_CYCLES" in a:
        w = a["SQ_WAVE_CYCLES"]
        print(f"  wait_any {a['SQ_WAIT_ANY']/w:.3f} wait_inst {a['SQ_WAIT_INST_ANY']/w:.3f} active {a['SQ_ACTIVE_INST_ANY']/w:.3f}")

if len(sys.argv) > 2:
    p = js["passes"]
    if all("mfma_busy" in p.get(k, {}) and "engine_us" in p.get(k, {}) for k in ("fwd", "bwd")):
        t = p["fwd"]["engine_us"] + p["bwd"]["engine_us"]
        js["engines_mfma_busy"] = round((p["fwd"]["mfma_busy"] * p["fwd"]["engine_us"] +
                                         p["bwd"]["mfma_busy"] * p["bwd"]["engine_us"]) / t, 4)
    js["definition"] = ("SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) per engine kernel "
                        "(profiled passes run at a lower clock); engines_mfma_busy weights the two by duration")
    json.dump(js, open(sys.argv[2], "w"), indent=1)
