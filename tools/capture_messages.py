"""Print the exception messages this stack raises for calls refused inside HIP graph capture
(collectives on gloo / RCCL, host syncs), as JSON lines, and whether TrainStep's classifier
(`train_step._is_capture_error`) takes each for a capture error.  Run on the GPU box; the
messages feed tests/test_host_cpu.py::test_capture_error_messages."""
import json
import os
import socket
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from twotower_amd.train_step import _is_capture_error  # noqa: E402


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def attempt(name, fn):
    dev = torch.device("cuda", 0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    msg = None
    try:
        with torch.cuda.graph(g):
            fn(dev)
    except Exception as e:  # noqa: BLE001 - we want every message
        msg = f"{type(e).__name__}: {e}"
    try:
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001
        msg = (msg or "") + f" | after: {e}"
    print(json.dumps({"case": name, "message": msg, "classified_capture": None if msg is None else _is_capture_error(
        RuntimeError(msg))}), flush=True)


def main(backend):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    torch.cuda.set_device(0)
    if backend:
        dist.init_process_group(backend, rank=0, world_size=1, device_id=torch.device("cuda", 0) if backend == "nccl" else None)
    x = torch.ones(64, device="cuda:0")
    if backend:
        attempt(f"{backend} all_to_all_single", lambda d: dist.all_to_all_single(torch.empty_like(x), x))
        attempt(f"{backend} all_gather_into_tensor", lambda d: dist.all_gather_into_tensor(torch.empty_like(x), x))
        attempt(f"{backend} all_reduce", lambda d: dist.all_reduce(x))
        dist.destroy_process_group()
    else:
        attempt("item()", lambda d: x.sum().item())
        attempt("torch.cuda.synchronize()", lambda d: torch.cuda.synchronize())
        attempt("cpu copy", lambda d: x.cpu())
        ev = torch.cuda.Event()

        def q(d):
            ev.record()
            ev.query()
        attempt("event.query()", q)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "")
