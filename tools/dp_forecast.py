"""Forecast of the N-rank step (N = 2, 4, 8 on one 8 x MI355X node) from one-GPU measurements and an
assumed RCCL rate: what bounds >= 6x scaling, per workload and table exchange.

Inputs (all measured on one GPU, committed under profiles/):
  --step-ms      C3, C4 (pairs form) and C5 one-GPU step times (bench.py, ms)
  --update-ms    the one-GPU fused table update of each (the op the exchange replaces, ms)
  --table-sync   tools/mb.py table_sync output (JSON lines, c3 and c5): per-rank GPU work of the
                 gather / shard / owner exchanges at N ranks, and their link bytes per rank
  --scorer-dp    tools/mb.py scorer_dp output (JSON lines): one rank's scorer passes at the N-rank
                 shapes of C4's triplet form (M = N 2B); the pairs form (M = N B) is read at half
                 the candidates
Link model: a collective moving X bytes into each rank takes X / bw, bw = the per-rank RCCL
all-gather / reduce-scatter rate (xGMI: 7 links x 153.6 GB/s bidirectional = 537.6 GB/s per direction
per GPU; RCCL reaches 60-80 % of that on large messages, so 320-430 GB/s, given as --bw).  Exposed
link time is what cannot overlap: the table exchange sits between the backward and the next forward
(twotower/train.py:138-139), minus the chunk pipeline's overlap with the update work itself.
Column exchange (--column, tools/mb.py column_sync): per rank the one-GPU step minus its own gather and
table update, plus the column gather of every rank's sequences from the (V, E/N) slab, the two layout
copies, the merged-plan slab update, and the exposed links: the ids all-gather before the gather, the
pooled all-to-all after it and the gs all-to-all after the backward (the plan all-gather runs on the
plan's stream beside the towers and the loss, and is not charged).
Usage: python tools/dp_forecast.py --table-sync c3.jsonl c5.jsonl --scorer-dp dp.jsonl [--column col.jsonl]
       [--bw 320 430]"""
import argparse
import json


def load(paths):
    out = []
    for p in paths:
        for ln in open(p):
            ln = ln.strip()
            if ln.startswith("{"):
                out.append(json.loads(ln))
    return out


def exch(mode, r, bw_gbs):
    """(GPU work us, exposed link us) of one table exchange per rank and step."""
    link_us = r["link_MB_per_rank"][mode] * 1e6 / (bw_gbs * 1e9) * 1e6
    # the one-GPU step already holds its own plan (plan_own_us): gather and owner sort every rank's
    # tokens instead, counted here as exposed (the plan runs on a side stream beside the forward)
    if mode == "gather":  # factored all-gather (overlaps nothing: it follows the backward), then the
        work = r["gather_update_us"] + r["plan_all_ranks_us"] - r["plan_own_us"]  # replicated update
        return work, link_us
    if mode == "shard":  # dense gradient, then per chunk: reduce-scatter -> AdamW(own) -> all-gather,
        work = r["shard_dense_grad_us"] + r["shard_adamw_us"]  # pipelined behind the next chunk's rows
        return work, max(0.0, link_us - r["shard_dense_grad_us"] * 7 / 8)
    # owner: factored all-gather (exposed), then per chunk: own-row update -> row all-gather (pipelined)
    ag_factored = (r["link_MB_per_rank"]["gather"]) * 1e6 / (bw_gbs * 1e9) * 1e6
    ag_rows = link_us - ag_factored
    work = r["owner_update_us"]
    return work + r["owner_plan_us"] - r["plan_own_us"], ag_factored + max(0.0, ag_rows - work * 7 / 8)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--table-sync", nargs="+", required=True)
    ap.add_argument("--scorer-dp", default=None)
    ap.add_argument("--step-ms", nargs=3, type=float, default=[0.857, 0.672, 1.90], metavar=("C3", "C4P", "C5"))
    ap.add_argument("--update-ms", nargs=3, type=float, default=[0.276, 0.276, 1.211], metavar=("C3", "C4P", "C5"))
    ap.add_argument("--bw", nargs="+", type=float, default=[320.0, 430.0])
    ap.add_argument("--column", nargs="*", default=[])
    a = ap.parse_args()
    ts = load(a.table_sync)
    sdp = {r["world"]: r for r in load([a.scorer_dp])} if a.scorer_dp else {}
    rows = []
    for cfg, step, upd in (("c5", a.step_ms[2], a.update_ms[2]), ("c3", a.step_ms[0], a.update_ms[0]),
                           ("c4p", a.step_ms[1], a.update_ms[1])):
        table = "c5" if cfg == "c5" else "c3"
        base = step - upd  # everything but the table update, per rank (weak scaling: constant for C5)
        for r in (x for x in ts if x["config"] == table and x["ranks"] > 1):
            N = r["ranks"]
            extra_scorer = 0.0
            if cfg in ("c3", "c4p") and sdp:
                # cross-device negatives: each rank's scorer work grows with N (global negatives)
                w1 = sdp[1]["fwd_us"] + sdp[1]["bwd_us"]
                key = N if cfg == "c3" else N // 2  # pairs form: N B candidates = the triplet shape at N / 2
                if key in sdp:
                    extra_scorer = (sdp[key]["fwd_us"] + sdp[key]["bwd_us"] - (w1 if cfg == "c3" else
                                    (sdp[1]["fwd_us"] + sdp[1]["bwd_us"]) / 2)) / 1e3
                else:  # N = 1 pairs shape (M = B): half of the triplet shape's work
                    extra_scorer = 0.0
            for mode in ("gather", "shard", "owner"):
                for bw in a.bw:
                    work, link = exch(mode, r, bw)
                    t = base + extra_scorer + (work + link) / 1e3
                    rows.append((cfg, N, mode, bw, round(t, 3), round(N * step / t, 2)))
    def scorer_growth(cfg, N):
        """Extra per-rank scorer ms at N ranks (global negatives): the N-rank shape's passes minus the
        one-GPU shape's, from tools/mb.py scorer_dp (the triplet form's M = N 2B; the pairs form's
        M = N B is the triplet shape at N / 2, and its one-GPU shape half the triplet's)."""
        if not sdp:
            return 0.0
        w1 = sdp[1]["fwd_us"] + sdp[1]["bwd_us"]
        key = N if cfg == "c3" else N // 2
        return (sdp[key]["fwd_us"] + sdp[key]["bwd_us"] - (w1 if cfg == "c3" else w1 / 2)) / 1e3

    for r in load(a.column) if a.column else []:
        N = r["ranks"]
        if N < 2:
            continue
        cfg = r["config"]
        zipf = r.get("zipf")
        step, upd = (a.step_ms[2], a.update_ms[2]) if cfg == "c5" else (a.step_ms[0], a.update_ms[0])
        work = (r["col_gather_us"] - r["gather_own_us"] + r["permute_pooled_us"] + r["permute_grad_us"]
                + r["col_update_us"])
        mb = r["link_MB_per_rank"]
        exposed_mb = mb["ids_allgather"] + mb["pooled_alltoall"] + mb["grad_alltoall"]
        # C5 and C3 with per-sample losses (no cross-rank term); the in-batch loss the driver scales
        # (bench.py --gpus N at C3: the triplet form, M = N 2B) and C4's pairs form (M = N B) add the
        # per-rank scorer growth of global negatives (its candidate all-gather overlaps the local
        # launch of the two-launch forward and is not charged)
        forms = [("c5" + (f" (Zipf {zipf} ids)" if zipf else ""), step, upd, 0.0)] if cfg == "c5" else [
            ("c3 (per-sample losses)", step, upd, 0.0),
            ("c3 in-batch, M = N 2B (bench --gpus N)", step, upd, scorer_growth("c3", N)),
            ("c4 pairs, M = N B", a.step_ms[1], a.update_ms[1], scorer_growth("c4p", N))]
        for label, st, up, extra in forms:
            if extra is None:
                continue
            for bw in a.bw:
                t = st - up + extra + (work + exposed_mb * 1e6 / (bw * 1e9) * 1e6) / 1e3
                rows.append((label, N, "column", bw, round(t, 3), round(N * st / t, 2)))
    print("| workload | N | table exchange | RCCL GB/s per rank | forecast ms/step | speedup vs 1 GPU |")
    print("|---|---|---|---|---|---|")
    for cfg, N, mode, bw, t, s in rows:
        print(f"| {cfg} | {N} | {mode} | {bw:.0f} | {t} | {s} |")


if __name__ == "__main__":
    main()
