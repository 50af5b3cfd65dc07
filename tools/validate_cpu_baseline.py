"""Cross-check of the CPU baseline: oracle/cpu_step.py, the torch-CPU
restatement bench.py times on the GPU box's host as `cpu_baseline`, against the REFERENCE's own
training loop, twotower.train.train_epoch (twotower/train.py:64-207), on the same cores, the same
batches and the same model shapes.  Run in the build container only (it imports /root/reference
through the namespace stub tests/golden/make_golden.py uses; wandb / twotower.huggingface are
stubbed and never called):

    python tools/validate_cpu_baseline.py [--threads N] [--out profiles/r02_cpu_baseline_validation.json]

Cases: C1 (configs/char_tower.yml: char vocab 34, E 64, H 128, tied, triplet m 0.2, batch 64,
L 64) and the C3 shape (V 200k, E = H 256, L 64, batch 8192, in-batch loss over cat[p, n]).  The
reference loop also computes per-batch cosine monitors, .item() calls and a tqdm bar
(train.py:143-166); those are part of its step time.  Pass: the port's pairs/s within 15 % of the
reference's.
"""
import argparse
import importlib
import json
import os
import sys
import time
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF = "/root/reference"

from oracle.cpu_step import host_cores, ref_loss, time_cpu_step  # noqa: E402
import twotower_amd as tt  # noqa: E402


def load_reference():
    for pkg in ("twotower", "dataset_factory"):
        m = types.ModuleType(pkg)
        m.__path__ = [os.path.join(REF, pkg)]
        sys.modules[pkg] = m
    hf = types.ModuleType("twotower.huggingface")
    hf.save_and_upload = None
    sys.modules["twotower.huggingface"] = hf
    sys.modules["wandb"] = types.ModuleType("wandb")
    return {n: importlib.import_module(f"twotower.{n}") for n in ("embeddings", "encoders", "losses", "train")}


def time_reference(R, V, E, H, batches, loss, steps):
    torch.manual_seed(0)
    emb = R["embeddings"].build("lookup", vocab_size=V, embedding_dim=E)
    model = R["encoders"].build_two_tower("mean", emb, hidden_dim=H, tied_weights=True)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    if loss == "triplet":
        loss_fn = R["losses"].build("triplet", margin=0.2)
    else:  # the reference's in-batch loss on cat[p, n] (its own function; train.py:133 cannot call it)
        ib = R["losses"].in_batch_sampled_softmax_loss

        def loss_fn(q, p, n):
            return ib(q, torch.cat([p, n]), 0.1)
    R["train"].train_epoch(model, batches[:1], opt, loss_fn, "cpu")  # warm-up
    data = [batches[k % len(batches)] for k in range(steps)]
    t0 = time.perf_counter()
    R["train"].train_epoch(model, data, opt, loss_fn, "cpu")
    dt = time.perf_counter() - t0
    return {"pairs_per_s": sum(b[0].shape[0] for b in data) / dt, "steps": steps, "seconds": dt}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=None)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_cpu_baseline_validation.json"))
    args = ap.parse_args()
    if args.threads:
        torch.set_num_threads(args.threads)
    R = load_reference()
    import logging
    logging.disable(logging.WARNING)
    cases = [
        ("C1", dict(V=34, E=64, H=128, B=64, L=64, loss="triplet", steps=1500)),
        ("C3", dict(V=200_000, E=256, H=256, B=8192, L=64, loss="in_batch", steps=5)),
    ]
    out = {"host": host_cores(), "cases": {}}
    for name, c in cases:
        batches = [tuple(t.long() for t in tt.data.synthetic_triplets(c["B"], c["L"], c["V"], seed=k, device="cpu"))
                   for k in range(2)]
        ref = time_reference(R, c["V"], c["E"], c["H"], batches, c["loss"], c["steps"])
        port = time_cpu_step(c["V"], c["E"], c["H"], batches, loss=c["loss"], min_seconds=1e9, max_steps=c["steps"])
        ratio = port["pairs_per_s"] / ref["pairs_per_s"]
        out["cases"][name] = {"shape": c, "reference_train_epoch": ref, "port": port, "port_over_reference": ratio,
                              "within_15pct": abs(ratio - 1) <= 0.15}
        print(name, json.dumps(out["cases"][name]), flush=True)
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
