"""Run under torch.distributed.run (gloo, CPU) by test_distributed_cpu.py: every rank builds
bench.child_world_env() and starts a child that forms its own gloo world of the same ranks with
it and all-reduces its rank; the parent prints "rank r child ok" when its child reported the sum."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] == "child":
    dist.init_process_group("gloo", rank=int(os.environ["RANK"]), world_size=int(os.environ["WORLD_SIZE"]))
    t = torch.tensor([dist.get_rank() + 1])
    dist.all_reduce(t)
    print(f"child sum {int(t.item())}", flush=True)
    dist.destroy_process_group()
    sys.exit(0)

import bench  # noqa: E402

dist.init_process_group("gloo")
env = bench.child_world_env(torch.device("cpu"))
r = subprocess.run([sys.executable, os.path.abspath(__file__), "child"], env=env, capture_output=True, text=True,
                   timeout=120)
world = dist.get_world_size()
want = f"child sum {world * (world + 1) // 2}"
ok = r.returncode == 0 and want in r.stdout
print(f"rank {dist.get_rank()} child {'ok' if ok else 'failed: ' + r.stdout + r.stderr[-500:]}", flush=True)
dist.destroy_process_group()
