"""Host-side checks that need no GPU: the C-ABI library loads and exports every symbol the public
header declares, its argument validation answers without touching a device, and the Python
surface mirrors the reference's plugin API (registries, builders and their errors, parameter
names, install() into a reference-shaped package, packed-view detection)."""
import ctypes
import os
import subprocess
import sys
import types

import pytest
import torch

import twotower_amd as tt
from twotower_amd import _lib, losses


# ---------------------------------------------------------------------------------------------
# C ABI
def test_library_exports_every_header_symbol():
    lib = _lib.lib()
    names = _lib.header_symbols()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    # the ctypes table binds exactly the declared functions
    assert sorted(_lib._SIGNATURES) == names
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True)
    exported = {ln.split()[-1] for ln in out.stdout.splitlines() if " T " in ln}
    assert set(names) <= exported
    assert lib.tt_version() == 1


def test_library_is_gfx950_only():
    """Every offload bundle embedded in the library targets gfx950 (no other ISA, no fallback)."""
    import re

    blob = open(_lib.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets


@pytest.mark.parametrize("call,msg", [
    (lambda L: L.tt_bag_mean_fwd(None, 0, 64, None, 0, 1, 4, 4, None, None, None), "V=0"),
    (lambda L: L.tt_bag_mean_fwd(None, 10, 64, None, 7, 1, 4, 4, None, None, None), "ids_dtype"),
    (lambda L: L.tt_bag_mean_fwd(None, 10, 64, None, 0, 2, 4, 3, None, None, None), "bad ids shape"),
    (lambda L: L.tt_adamw(None, None, None, None, 16, 1e-3, 0.9, 0.999, 1e-8, 0.01, 0, None), "step must be"),
    (lambda L: L.tt_adamw_multi(None, 17, None), "count=17"),
    (lambda L: L.tt_adamw_multi_ex(None, None, 17, None, 0, 1e-3, 0.9, 0.999, 1e-8, 0.01, None, None), "count=17"),
    (lambda L: L.tt_adamw_multi_ex(None, None, 0, None, 2, 1e-3, 0.9, 0.999, 1e-8, 0.01, None, None),
     "needs slots and a ticket"),
    (lambda L: L.tt_pack_blocks(None, None, 9, None, None), "count=9"),
    (lambda L: L.tt_head_wgrad2_parts(64, 0, ctypes.byref(ctypes.c_int64()), ctypes.byref(ctypes.c_int64())),
     "tt_head_wgrad2_parts: N=64"),
    (lambda L: L.tt_colsum(ctypes.c_void_p(16), 8, 6, ctypes.c_void_p(16), ctypes.c_void_p(16), 1 << 20, None), "cols % 4"),
    (lambda L: L.tt_inbatch_fwd(None, None, 8, 4, 64, 0, 10.0, 0, 1, None, None, None, None, None, 0, None),
     "label"),
])
def test_validation_without_a_device(call, msg):
    rc = call(_lib.lib())
    assert rc != 0
    assert msg in _lib.last_error(), _lib.last_error()


def test_ops_refuse_cpu_tensors():
    w = torch.zeros(10, 4)
    ids = torch.ones(2, 3, dtype=torch.int64)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        tt.ops.bag_mean_pool(w, ids)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        tt.ops.in_batch_softmax_loss(torch.zeros(2, 64), torch.zeros(4, 64))


# ---------------------------------------------------------------------------------------------
# plugin surface (twotower/embeddings.py:159-181, encoders.py:228-272, losses.py:122-150)
def test_registries_and_builder_errors():
    assert set(tt.embeddings.REGISTRY) == {"lookup", "word2vec", "glove"}
    assert set(tt.TOWER_REGISTRY) == {"mean", "avg_pool"}
    assert set(tt.LOSS_REGISTRY) == {"triplet", "multiple_negatives", "in_batch"}
    with pytest.raises(ValueError, match=r"Unknown embedding: nope\. Available options: \['lookup'"):
        tt.embeddings.build("nope", vocab_size=10)
    with pytest.raises(ValueError, match=r"Unknown tower architecture: nope\. Available options"):
        tt.build_tower("nope", tt.embeddings.build("lookup", vocab_size=10, embedding_dim=8))
    with pytest.raises(ValueError, match=r"Unknown loss function: nope\. Available options"):
        losses.build("nope")
    f = losses.build("triplet", margin=0.3)
    assert f.func is losses.contrastive_triplet_loss and f.keywords == {"margin": 0.3}
    assert losses.build("in_batch") is losses.in_batch_sampled_softmax_loss
    with pytest.raises(ImportError):
        tt.embeddings.build("glove", vocab_size=10, embedding_dim=8)


def test_lookup_embedding_layout_and_state_dict_names():
    emb = tt.embeddings.build("lookup", vocab_size=50, embedding_dim=8)
    assert (emb.vocab_size, emb.embedding_dim, emb.padding_idx) == (50, 8, 0)
    assert isinstance(emb.embedding, torch.nn.Embedding) and emb.embedding.padding_idx == 0
    assert torch.equal(emb.embedding.weight[0], torch.zeros(8))  # nn.Embedding zeroes the padding row
    model = tt.build_two_tower("mean", emb, hidden_dim=16, tied_weights=True)
    keys = sorted(model.state_dict())
    tower = ["embedding.embedding.weight", "feed_forward.0.bias", "feed_forward.0.weight", "feed_forward.2.bias",
             "feed_forward.2.weight"]
    assert keys == sorted([f"query_tower.{k}" for k in tower] + [f"document_tower.{k}" for k in tower])
    assert model.document_tower is model.query_tower
    untied = tt.build_two_tower("mean", emb, hidden_dim=16, tied_weights=False)
    assert untied.document_tower is not untied.query_tower
    assert untied.document_tower.embedding is untied.query_tower.embedding  # one shared table (encoders.py:265,270)
    avg = tt.build_tower("avg_pool", emb, hidden_dim=16)
    assert sorted(k for k in avg.state_dict() if k.startswith("projection")) == [
        "projection.0.bias", "projection.0.weight", "projection.2.bias", "projection.2.weight"]


def test_optimizer_state_dict_interchanges_with_torch():
    p = [torch.nn.Parameter(torch.randn(4, 4)), torch.nn.Parameter(torch.randn(4))]
    ref = torch.optim.AdamW(p, lr=1e-3)
    for x in p:
        x.grad = torch.ones_like(x)
    ref.step()
    mine = tt.optim.AdamW(p, lr=1e-3, capturable=True)
    mine.load_state_dict(ref.state_dict())
    st = mine.state[p[0]]
    assert set(st) == {"step", "exp_avg", "exp_avg_sq"} and float(st["step"]) == 1.0
    assert mine.param_groups[0]["capturable"] is True
    # and back: torch reads ours
    ref2 = torch.optim.AdamW(p, lr=1e-3)
    ref2.load_state_dict(mine.state_dict())
    assert torch.equal(ref2.state[p[0]]["exp_avg"], st["exp_avg"])


def test_install_into_reference_shaped_package():
    pkg = "fake_twotower_ref"
    mods = {}
    for sub in ("", ".embeddings", ".encoders", ".losses", ".train"):
        m = types.ModuleType(pkg + sub)
        mods[pkg + sub] = m
    mods[pkg].__path__ = []
    mods[pkg + ".embeddings"].REGISTRY = {"lookup": object}
    mods[pkg + ".encoders"].TOWER_REGISTRY = {"mean": object}
    mods[pkg + ".losses"].LOSS_REGISTRY = {"triplet": None}
    mods[pkg + ".train"].build_two_tower = None
    sys.modules.update(mods)
    try:
        tt.install(pkg)
        assert mods[pkg + ".embeddings"].REGISTRY["lookup"] is tt.LookupEmbedding
        assert mods[pkg + ".encoders"].TOWER_REGISTRY["mean"] is tt.MeanPoolingTower
        assert mods[pkg + ".encoders"].build_two_tower is tt.build_two_tower
        assert mods[pkg + ".train"].build_two_tower is tt.build_two_tower
        assert mods[pkg + ".losses"].LOSS_REGISTRY["in_batch"] is tt.in_batch_sampled_softmax_loss
    finally:
        for k in mods:
            sys.modules.pop(k, None)


def test_packed_view_detection():
    base = torch.randn(9, 4)
    q, p, n = torch.split(base, 3)
    assert losses._packed(q, p, n) is base
    assert losses._packed(q, n, p) is None           # out of order
    assert losses._packed(q, p) is None              # not the whole base
    assert losses._packed(q.clone(), p, n) is None   # not views of one tensor
    cand = losses._candidates(p, n)
    assert cand.data_ptr() == p.data_ptr() and cand.shape == (6, 4)


def test_synthetic_triplets_shape_and_padding():
    q, p, n = tt.data.synthetic_triplets(64, 16, 1000, seed=1, device="cpu")
    for t, (lo, hi) in ((q, (3, 12)), (p, (8, 16)), (n, (8, 16))):
        assert t.shape == (64, 16) and t.dtype == torch.int32
        lens = (t > 0).sum(1)
        assert int(lens.min()) >= lo and int(lens.max()) <= hi
        # trailing padding: no real token after the first pad
        pos = torch.arange(16)
        assert bool(((t > 0) == (pos < lens[:, None])).all())
        assert int(t.max()) < 1000
    assert tt.data.tokens_per_triplet(16) == pytest.approx(7.5 + 2 * 12)


# ---------------------------------------------------------------------------------------------
# checkpoints (twotower/utils.py:231-330; parameter layout pinned by tests/golden/state_dict.npz)
def _layout(golden):
    import json

    return json.loads(str(golden("state_dict")["layout_json"]))


def test_state_dict_layout_matches_reference(golden):
    L = _layout(golden)
    emb = tt.embeddings.build("lookup", vocab_size=50, embedding_dim=16)
    ours = {
        "mean_tied": tt.build_two_tower("mean", emb, hidden_dim=24, tied_weights=True),
        "mean_untied": tt.build_two_tower("mean", emb, hidden_dim=24, tied_weights=False),
        "avg_proj": tt.build_two_tower("avg_pool", emb, hidden_dim=24, tied_weights=True),
        "avg_noproj": tt.build_two_tower("avg_pool", emb, hidden_dim=16, tied_weights=True),
    }
    for k, m in ours.items():
        assert [[n, list(t.shape)] for n, t in m.state_dict().items()] == L[k], k
    m = ours["mean_tied"]
    opt = tt.optim.AdamW(m.parameters(), lr=1e-3)
    for p in m.parameters():
        p.grad = torch.ones_like(p)
        opt._state(p, False)  # materialise state without a kernel launch
    sd = opt.state_dict()
    assert sorted(sd["state"][0]) == L["optimizer"]["state_keys"]
    assert len(sd["state"]) == L["optimizer"]["n_state"]


def test_checkpoint_round_trip_reference_format(tmp_path):
    emb = tt.embeddings.build("lookup", vocab_size=30, embedding_dim=8)
    model = tt.build_two_tower("mean", emb, hidden_dim=12, tied_weights=True)
    ref_opt = torch.optim.AdamW(model.parameters(), lr=1e-3)
    for p in model.parameters():
        p.grad = torch.randn_like(p)
    ref_opt.step()
    path = tt.checkpoint.save_checkpoint(model, {"<PAD>": 0, "a": 1}, ref_opt, epoch=3, loss=0.5,
                                         checkpoint_dir=str(tmp_path))
    assert os.path.exists(path) and os.path.exists(tmp_path / "best_model.pt")
    raw = torch.load(path, weights_only=True)
    assert set(raw) == {"model", "vocab", "epoch", "loss", "timestamp", "optimizer"}
    assert raw["epoch"] == 3 and raw["vocab"]["a"] == 1
    emb2 = tt.embeddings.build("lookup", vocab_size=30, embedding_dim=8)
    model2 = tt.build_two_tower("mean", emb2, hidden_dim=12, tied_weights=True)
    opt2 = tt.optim.AdamW(model2.parameters(), lr=1e-3, capturable=True)
    ck = tt.checkpoint.load_checkpoint(path, model2, opt2)
    assert ck["loss"] == 0.5
    for (n, a), b in zip(model.state_dict().items(), model2.state_dict().values()):
        assert torch.equal(a, b), n
    p0 = next(model2.parameters())
    assert torch.equal(opt2.state[p0]["exp_avg"], ref_opt.state[next(model.parameters())]["exp_avg"])


def test_bench_op_report_shapes():
    """bench.op_report on synthetic per-op times: the scorer entry with the operand prep in the
    head's normalise pass (tt_inbatch_fwd_prepped + tt_inbatch_l2_prep) and without it, the
    multiple-negatives workload, and the dominant-op roofline (no GPU: the report is pure host math)."""
    import bench

    def op(ms, calls=10):
        return {"calls": calls, "mean_ms": ms, "total_ms": ms * calls}

    base = {"tt_bag_mean_fwd": op(0.13), "tt_bag_mean_bwd_adamw_planned": op(0.27), "tt_bag_plan": op(0.15),
            "tt_inbatch_bwd": op(0.097), "tt_adamw_multi": op(0.008)}
    for extra, prep in (({"tt_inbatch_fwd": op(0.165)}, None),
                        ({"tt_inbatch_fwd_prepped": op(0.155), "tt_inbatch_l2_prep": op(0.013)}, 0.003)):
        kernels, roof = bench.op_report({**base, **extra}, 10, "c3", 1, "bf16", 848_000.0, 131_584, "stored",
                                        normalise=lambda: 0.010)
        sc = next(k for k in kernels if k["bound"] == "mfma")
        want = 0.097 + extra.get("tt_inbatch_fwd", extra.get("tt_inbatch_fwd_prepped"))["mean_ms"] + (prep or 0.0)
        assert abs(sc["mean_ms"] - want) < 1e-4 and 0 < sc["frac"] < 1
        assert ("operand_prep_in_head_normalise" in sc["pass_ms"]) == (prep is not None)
        assert roof["op"].startswith("embedding bag backward fused") and roof["unit"] == "GB/s"
    # the backward combine fused with the head's F.normalize backward: charged beyond a plain one
    fused = {k: v for k, v in base.items() if k != "tt_inbatch_bwd"}
    fused.update({"tt_inbatch_bwd_l2": op(0.100), "tt_inbatch_fwd_prepped": op(0.155)})
    kernels, _ = bench.op_report(fused, 10, "c3", 1, "bf16", 848_000.0, 131_584, "stored",
                                 l2_backward=lambda: 0.012)
    sc = next(k for k in kernels if k["bound"] == "mfma")
    assert sc["abi"] == "tt_inbatch_fwd_prepped+tt_inbatch_bwd_l2" and abs(sc["mean_ms"] - (0.155 + 0.088)) < 1e-4
    assert sc["pass_ms"]["plain_l2_backward_subtracted"] == 0.012
    kernels, roof = bench.op_report({"tt_bag_mean_fwd": op(0.34), "tt_multi_neg_fwd": op(0.026),
                                     "tt_multi_neg_bwd": op(0.031)}, 10, "c5", 1, "fp32", 2.0e6, 131_584, "stored")
    assert {k["abi"] for k in kernels} == {"tt_bag_mean_fwd", "tt_multi_neg_fwd", "tt_multi_neg_bwd"}


# messages this stack raised for calls refused under HIP graph capture (tools/capture_messages.py on
# an MI355X box, torch 2.10 + ROCm 7: gloo collectives on GPU tensors, host syncs); RCCL collectives
# capture without error
_SEEN_CAPTURE_MESSAGES = [
    "HIP error: operation failed due to a previous error during capture\nSearch for "
    "`hipErrorStreamCaptureInvalidated' in https://rocm.docs.amd.com/projects/HIP/en/latest/index.html",
    "Cannot register the state during capturing stage. during CUDA graph capture. If you need this call to be "
    "captured, please file an issue. Current hipStreamCaptureStatus: hipStreamCaptureStatusInvalidated",
    "hipErrorStreamCaptureUnsupported: operation not permitted when stream is capturing",
    "CUDA error: operation not permitted when stream is capturing",
    "hipErrorCapturedEvent: operation not permitted on an event last recorded in a capturing stream",
    # torch.cuda.graph's capture_end after another thread's refused query invalidated a global-mode
    # capture (profiles/r07t_capture_poll_probe.txt)
    "status == hipStreamCaptureStatus::hipStreamCaptureStatusActive INTERNAL ASSERT FAILED at "
    "\"/pytorch/aten/src/ATen/hip/HIPGraph.cpp\":116, please report a bug to PyTorch. ",
]


def test_capture_error_messages():
    """TrainStep falls back to eager only for capture refusals; these are the messages
    actually seen on this stack, and errors of the step itself stay fatal."""
    from twotower_amd.train_step import _is_capture_error

    for m in _SEEN_CAPTURE_MESSAGES:
        assert _is_capture_error(RuntimeError(m)), m
    for m in ("tt_inbatch_fwd: workspace too small: need 10 have 5", "CUDA out of memory. Tried to allocate 2.00 GiB",
              "HIP error: an illegal memory access was encountered", "Expected all tensors to be on the same device",
              "NCCL error: unhandled system error"):
        assert not _is_capture_error(RuntimeError(m)), m
