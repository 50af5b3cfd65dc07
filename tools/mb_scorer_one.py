"""One scorer configuration, few iterations (for counter collection)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from twotower_amd import ops, _lib
if len(sys.argv) > 5:  # a variant library (tools/build_variants.sh)
    _lib.LIB_PATH = os.path.abspath(sys.argv[5])
B, M, H = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
dt = sys.argv[4] if len(sys.argv) > 4 else "bf16"
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.nn.functional.normalize(torch.randn(B, H, device="cuda", generator=g), dim=-1).requires_grad_(True)
d = torch.nn.functional.normalize(torch.randn(M, H, device="cuda", generator=g), dim=-1).requires_grad_(True)
for _ in range(3):
    ops.in_batch_softmax_loss(q, d, 0.1, compute_dtype=dt).backward()
torch.cuda.synchronize()
