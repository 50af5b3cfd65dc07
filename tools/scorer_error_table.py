"""Measured error of the in-batch scorer forms (GPU; not a test).

For each shape and compute form, the max-abs-normalised error of loss, dq and dd against a float64
computation of in_batch_sampled_softmax_loss (twotower/losses.py:88-118) on
  * the bf16-rounded operands the bf16 forms score ("rounded"), and
  * the original fp32 operands ("fp32 in": what the reference itself would compute).
The test tolerances in tests/test_gpu_kernels.py and tests/test_gpu_fullsize.py are set from this
table (about 1.5x the largest measured figure per form).  Prints one JSON line per case.

python tools/scorer_error_table.py [--big]   (--big adds C3 and the C4 per-rank shape)
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from twotower_amd import ops  # noqa: E402

DEV = "cuda"


def ref64(q, d, tau, off, g):
    z = (q.double() @ d.double().T) / tau
    B = q.shape[0]
    lab = torch.arange(B, device=DEV) + off
    lse = torch.logsumexp(z, 1)
    loss = (lse - z[torch.arange(B, device=DEV), lab]).mean()
    P = torch.exp(z - lse[:, None])
    del z
    P[torch.arange(B, device=DEV), lab] -= 1.0
    P *= g / B
    dq = P @ d.double() / tau
    dd = P.T @ q.double() / tau
    return loss.item(), dq, dd


def rel(a, b):
    return float((a.double() - b).abs().max() / b.abs().max().clamp_min(1e-300))


def run(B, M, H, off, form, seed):
    gen = torch.Generator(device=DEV).manual_seed(seed)
    q = torch.nn.functional.normalize(torch.randn(B, H, device=DEV, generator=gen), dim=-1)
    d = torch.nn.functional.normalize(torch.randn(M, H, device=DEV, generator=gen), dim=-1)
    dt, bwd = {"bf16_stored": ("bf16", "stored"), "bf16_recompute": ("bf16", "recompute"),
               "bf16_split": ("bf16_split", "stored"), "fp32": ("fp32", "stored")}[form]
    prev = ops.set_inbatch_backward(bwd)
    Q, D = q.clone().requires_grad_(True), d.clone().requires_grad_(True)
    g = 0.7
    loss = ops.InBatchSoftmaxLoss.apply(Q, D, 10.0, off, dt, None)
    loss.backward(torch.tensor(g, device=DEV))
    torch.cuda.synchronize()
    ops.set_inbatch_backward(prev)
    out = {"B": B, "M": M, "H": H, "off": off, "form": form}
    for tag, (qq, dd_) in (("rounded", (q.bfloat16().float(), d.bfloat16().float())), ("fp32_in", (q, d))):
        if tag == "rounded" and dt == "fp32":
            continue
        rl, rdq, rdd = ref64(qq, dd_, 0.1, off, g)
        out[tag] = {"loss": abs(loss.item() - rl) / abs(rl), "dq": rel(Q.grad, rdq), "dd": rel(D.grad, rdd)}
        del rdq, rdd
    torch.cuda.empty_cache()
    return out


def test_shapes():
    """Every (B, M, H, off) the GPU tests run the bf16 forms at, three seeds each: the per-form
    maxima set BF16_GRAD_TOL / BF16_SPLIT_GRAD_TOL in tests/test_gpu_kernels.py."""
    cases = [(B, M, H, off) for H in (32, 64, 128, 256)
             for (B, M, off) in [(300, 700, 0), (129, 129, 0), (64, 256, 128), (1000, 2000, 1000), (1, 64, 0),
                                 (320, 330, 10), (448, 900, 0), (2500, 2600, 100)]]
    worst = {}
    for (B, M, H, off) in cases:
        for form in ("bf16_stored", "bf16_recompute", "bf16_split"):
            for seed in range(3):
                r = run(B, M, H, off, form, seed=1000 * seed + B + M + H)
                e = max(r["rounded"]["dq"], r["rounded"]["dd"])
                if e > worst.get(form, (0,))[0]:
                    worst[form] = (e, B, M, H, off, seed)
    print(json.dumps({"test_shapes_worst": worst}), flush=True)


def main():
    if "--tests" in sys.argv:
        return test_shapes()
    shapes = [(300, 700, H, 0) for H in (32, 64, 128, 256)] + [(1000, 2000, 256, 1000), (129, 129, 64, 0)]
    if "--big" in sys.argv:
        shapes += [(8192, 16384, 256, 0), (8192, 131072, 256, 5 * 16384), (4096, 8192, 128, 0)]
    for (B, M, H, off) in shapes:
        for form in ("bf16_stored", "bf16_recompute", "bf16_split", "fp32"):
            if form == "fp32" and B * M > 1 << 26:
                continue
            print(json.dumps(run(B, M, H, off, form, seed=B + M + H)), flush=True)


if __name__ == "__main__":
    main()
