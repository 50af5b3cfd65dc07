"""TrainStep's graph capture beside another thread that polls the device, as a process group's
watchdog does.  Under the default global capture mode HIP refuses another thread's stream query
while a capture runs ("operation not permitted when stream is capturing": the message the
ProcessGroupNCCL watchdog aborted with once in the one-rank RCCL graph test) and the capture is
invalidated; TrainStep captures in thread-local mode, where both go through
(tools/repro/capture_poll_probe.py, profiles/r07t_capture_poll_probe.txt: global + stream query
fails, thread-local passes; an event query passes in both)."""
import threading

import pytest
import torch

import twotower_amd as tt

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_capture_beside_a_polling_thread():
    V, E, B, L = 3000, 256, 128, 12
    torch.manual_seed(3)
    emb = tt.embeddings.build("lookup", vocab_size=V, embedding_dim=E)
    model = tt.build_two_tower("mean", emb, hidden_dim=E, tied_weights=True).to(DEV)
    opt = tt.optim.AdamW(model.parameters(), lr=1e-3, fused_tables=True, tables=[emb], capturable=True)
    step = tt.TrainStep(model, tt.losses.build("in_batch", temperature=0.1, compute_dtype="bf16"), opt,
                        graph=True, eager_steps=1)
    batches = [tt.data.synthetic_triplets(B, L, V, seed=k, device=DEV) for k in range(3)]
    torch.cuda.synchronize()
    stop, errors, polls = threading.Event(), [], [0]

    def poll():
        ps = torch.cuda.Stream()  # the polling thread's own stream, as a watchdog queries its work
        while not stop.is_set():
            try:
                ps.query()
                polls[0] += 1
            except Exception as e:  # noqa: BLE001 -- a refused poll is what this test looks for
                errors.append(repr(e))
                return

    th = threading.Thread(target=poll, daemon=True)
    th.start()
    try:
        losses = [float(step(*batches[k % 3])) for k in range(4)]  # step 2 captures, 3-4 replay
    finally:
        stop.set()
        th.join(timeout=10)
    assert not errors, errors
    assert polls[0] > 0
    assert step.graph, "the step fell back to eager"
    assert all(torch.isfinite(torch.tensor(losses))), losses
