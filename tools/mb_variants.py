"""A/B timing of library variants (tools/build_variants.sh) on the scorer at a given shape.

Each variant runs in its own process (one .so per process): forward and backward op times from HIP
events per ABI call (prep/engine/combine together), plus a loss/grad checksum against the first variant
so a variant that computes something else is flagged.  Usage:
  python tools/mb_variants.py [--shape B M H] [--dtype bf16] lib_a.so lib_b.so ...
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(lib, B, M, H, dt, iters):
    sys.path.insert(0, ROOT)
    from twotower_amd import _lib
    _lib.LIB_PATH = os.path.abspath(lib)
    import torch
    from twotower_amd import ops
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.nn.functional.normalize(torch.randn(B, H, device="cuda", generator=g), dim=-1).requires_grad_(True)
    d = torch.nn.functional.normalize(torch.randn(M, H, device="cuda", generator=g), dim=-1).requires_grad_(True)
    for _ in range(3):
        q.grad = d.grad = None
        loss = ops.in_batch_softmax_loss(q, d, 0.1, compute_dtype=dt)
        loss.backward()
    torch.cuda.synchronize()
    ck = [float(loss), float(q.grad.double().abs().sum()), float(d.grad.double().abs().sum())]
    _lib.TIMER.reset()
    _lib.TIMER.enabled = True
    for _ in range(iters):
        ops.in_batch_softmax_loss(q, d, 0.1, compute_dtype=dt).backward()
    _lib.TIMER.enabled = False
    s = _lib.TIMER.summary()
    f, b = s["tt_inbatch_fwd"]["mean_ms"] * 1e3, s["tt_inbatch_bwd"]["mean_ms"] * 1e3
    print(json.dumps({"lib": os.path.basename(lib), "fwd_us": round(f, 1), "bwd_us": round(b, 1),
                      "algo_pf": round(6 * B * M * H / ((f + b) * 1e-6) / 1e15, 3), "check": ck}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", nargs=3, type=int, default=[8192, 16384, 256])
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--child", default=None)
    ap.add_argument("libs", nargs="*")
    a = ap.parse_args()
    if a.child:
        return child(a.child, *a.shape, a.dtype, a.iters)
    ref = None
    for lib in a.libs:
        r = subprocess.run([sys.executable, __file__, "--child", lib, "--shape", *map(str, a.shape), "--dtype", a.dtype,
                            "--iters", str(a.iters)], capture_output=True, text=True, timeout=300)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode != 0 or not line:
            print(json.dumps({"lib": lib, "error": r.stderr[-800:]}), flush=True)
            if r.returncode in (-6, -11, 134, 139):
                sys.exit(1)  # a fault: start nothing more on the GPU
            continue
        res = json.loads(line[-1])
        if ref is None:
            ref = res["check"]
        res["check_rel"] = max(abs(x - y) / max(abs(y), 1e-30) for x, y in zip(res["check"], ref))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
