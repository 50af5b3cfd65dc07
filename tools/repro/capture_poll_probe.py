"""Probe: a graph capture beside a thread that polls (what a process group's watchdog does), in a
given capture mode.  Usage: python tools/repro/capture_poll_probe.py global|thread_local [what]
what: event (hipEventQuery on an event recorded before the capture), stream (hipStreamQuery on a
stream of the polling thread).  Prints one JSON line: whether the capture succeeded and what the
polling thread saw."""
import json
import sys
import threading

import torch

mode = sys.argv[1] if len(sys.argv) > 1 else "global"
what = sys.argv[2] if len(sys.argv) > 2 else "event"
x = torch.randn(1 << 20, device="cuda")
ev = torch.cuda.Event()
ev.record()
torch.cuda.synchronize()
stop, errors, polls = threading.Event(), [], [0]


def poll():
    ps = torch.cuda.Stream()
    while not stop.is_set():
        try:
            ev.query() if what == "event" else ps.query()
            polls[0] += 1
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e)[:200])
            return


th = threading.Thread(target=poll, daemon=True)
th.start()
ok, err = True, None
try:
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            y = x * 2 + 1  # warm up on the side stream
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g, capture_error_mode=mode):
        for _ in range(200):  # a capture long enough for the thread to poll during it
            y = y * 1.0001 + 1
    g.replay()
    torch.cuda.synchronize()
except Exception as e:  # noqa: BLE001
    ok, err = False, repr(e)[:200]
stop.set()
th.join(timeout=10)
print(json.dumps({"mode": mode, "what": what, "capture_ok": ok, "capture_error": err, "poll_errors": errors[:1],
                  "polls": polls[0]}), flush=True)
