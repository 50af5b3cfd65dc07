"""CPU: the drop-in, proven against the reference's own modules (not a stand-in package).

The reference's `twotower` package is loaded from /root/reference through a namespace stub (its
__init__ needs wandb; train.py imports wandb and twotower.huggingface, stubbed as empty modules
and never called), exactly as tests/golden/make_golden.py loads it.  Then
`twotower_amd.install("twotower")` runs, and the reference's own `build_pipeline`
(twotower/train.py:298-371) builds the pipeline from its own configs/char_tower.yml:
  * the tokeniser, TripletDataset and torch.optim.AdamW stay the reference's;
  * the embedding, the towers, the TwoTower model and the loss must come out as the HIP classes;
  * the loss must accept train.py:133's `loss_fn(q_vec, p_vec, n_vec)` call for every registry
    entry (triplet, in_batch, multiple_negatives), and the state_dict keys must be the
    reference model's.
The reference is absent on the GPU box: these tests skip there.  Nothing here runs a kernel.
"""
import importlib
import inspect
import os
import sys
import types

import pytest
import torch

REF = "/root/reference"
pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "twotower")), reason="reference not present")

@pytest.fixture()
def ref_pkg():
    saved = {k: sys.modules.get(k) for k in list(sys.modules) if k == "wandb" or k.split(".")[0] in
             ("twotower", "dataset_factory")}
    for k in saved:
        sys.modules.pop(k, None)
    for pkg in ("twotower", "dataset_factory"):
        m = types.ModuleType(pkg)
        m.__path__ = [os.path.join(REF, pkg)]
        sys.modules[pkg] = m
    hf = types.ModuleType("twotower.huggingface")
    hf.save_and_upload = None  # train.py:27 binds it; never called without a hub push
    sys.modules["twotower.huggingface"] = hf
    sys.modules["wandb"] = types.ModuleType("wandb")
    mods = {n: importlib.import_module(f"twotower.{n}") for n in ("embeddings", "encoders", "losses", "utils")}
    yield mods
    for k in [k for k in sys.modules if k == "wandb" or k.split(".")[0] in ("twotower", "dataset_factory")]:
        sys.modules.pop(k, None)
    sys.modules.update({k: v for k, v in saved.items() if v is not None})


def _triplet_parquet(path, n=48):
    import pandas as pd

    rows = [(f"what is item {i}", f"item {i} is a thing number {i}", f"unrelated text {(i * 7) % n}")
            for i in range(n)]
    pd.DataFrame(rows, columns=["query", "positive_doc", "negative_doc"]).to_parquet(path)


def _config(ref, data, **over):
    cfg = ref["utils"].load_config(os.path.join(REF, "configs", "char_tower.yml"))
    cfg["data"] = str(data)
    for k, v in over.items():  # a loss block is replaced whole (its kwargs go to the loss)
        cfg[k] = dict(v) if k == "loss" else {**cfg.get(k, {}), **v}
    return cfg


@pytest.mark.parametrize("install_before_train_import", [True, False])
def test_install_makes_reference_build_pipeline_produce_hip_classes(ref_pkg, tmp_path, install_before_train_import):
    import twotower_amd as tt

    if install_before_train_import:
        tt.install("twotower")
        train = importlib.import_module("twotower.train")
    else:  # train.py already imported: its bound build_two_tower is patched too
        train = importlib.import_module("twotower.train")
        tt.install("twotower")
    data = tmp_path / "triplets.parquet"
    _triplet_parquet(data)
    model, dataset, optimizer, loss_fn = train.build_pipeline(_config(ref_pkg, data), device="cpu")

    assert type(model) is tt.TwoTower
    assert type(model.query_tower) is tt.MeanPoolingTower and model.document_tower is model.query_tower
    assert type(model.query_tower.embedding) is tt.LookupEmbedding
    assert model.query_tower.embedding.vocab_size == dataset.vocab_size
    assert type(optimizer) is torch.optim.AdamW                       # train.py:359, unchanged
    assert getattr(loss_fn, "func", loss_fn) is tt.contrastive_triplet_loss
    assert loss_fn.keywords == {"margin": 0.2}                        # char_tower.yml loss block

    # state_dict keys (checkpoints, utils.py:272) equal the reference model's own
    ref_enc, ref_emb = ref_pkg["encoders"], ref_pkg["embeddings"]
    ref_model = ref_enc.TwoTower(ref_enc.MeanPoolingTower(ref_emb.LookupEmbedding(dataset.vocab_size, 64), 128),
                                 None, tied_weights=True)
    assert list(model.state_dict()) == list(ref_model.state_dict())
    for k, v in ref_model.state_dict().items():
        assert model.state_dict()[k].shape == v.shape, k

    # the DataLoader batches the reference feeds to model(q, p, n) (train.py:120-122)
    q, p, n = dataset[0]
    assert q.dtype == torch.long and q.shape == p.shape == n.shape


@pytest.mark.parametrize("loss_type,kw", [("triplet", {"margin": 0.2}), ("in_batch", {"temperature": 0.05}),
                                          ("multiple_negatives", {"temperature": 0.1})])
def test_every_registry_loss_binds_train_py_call(ref_pkg, tmp_path, loss_type, kw):
    import twotower_amd as tt

    tt.install("twotower")
    train = importlib.import_module("twotower.train")
    data = tmp_path / "triplets.parquet"
    _triplet_parquet(data)
    _, _, _, loss_fn = train.build_pipeline(_config(ref_pkg, data, loss={"type": loss_type, **kw}), device="cpu")
    assert getattr(loss_fn, "func", None) is tt.LOSS_REGISTRY[loss_type]
    assert loss_fn.keywords == kw
    v = torch.zeros(4, 8)
    inspect.signature(loss_fn).bind(v, v, v)                          # train.py:133


def test_avg_pool_and_untied_configs(ref_pkg, tmp_path):
    import twotower_amd as tt

    tt.install("twotower")
    train = importlib.import_module("twotower.train")
    data = tmp_path / "triplets.parquet"
    _triplet_parquet(data)
    cfg = _config(ref_pkg, data, encoder={"arch": "avg_pool", "tied_weights": False})
    model, _, _, _ = train.build_pipeline(cfg, device="cpu")
    assert type(model.query_tower) is tt.AveragePoolingTower and type(model.document_tower) is tt.AveragePoolingTower
    # one shared table even untied (encoders.py:265,270)
    assert model.query_tower.embedding is model.document_tower.embedding


def test_unknown_names_raise_the_reference_errors(ref_pkg):
    import twotower_amd as tt

    tt.install("twotower")
    with pytest.raises(ValueError, match="Unknown embedding"):
        ref_pkg["embeddings"].build("nope", vocab_size=10, embedding_dim=4)
    with pytest.raises(ValueError, match="Unknown tower architecture"):
        ref_pkg["encoders"].build_two_tower("nope", None, hidden_dim=4)
    with pytest.raises(ValueError, match="Unknown loss"):
        ref_pkg["losses"].build("nope")


@pytest.mark.parametrize("install_before_train_import", [True, False])
def test_config_opts_in_to_backward_table_update(ref_pkg, tmp_path, install_before_train_import):
    """`hip: {table_update: backward}` in an otherwise reference config (a namespace the reference
    never reads) makes the wrapped build_pipeline attach the fused table update to the loop's own
    torch.optim.AdamW; without it nothing changes; an unknown mode raises."""
    import twotower_amd as tt

    if install_before_train_import:
        tt.install("twotower")  # build_pipeline is wrapped when train.py is imported
        train = importlib.import_module("twotower.train")
    else:
        train = importlib.import_module("twotower.train")
        tt.install("twotower")
    assert getattr(train.build_pipeline, "_tt_wrapped", False)
    data = tmp_path / "triplets.parquet"
    _triplet_parquet(data)
    model, _, optimizer, _ = train.build_pipeline(_config(ref_pkg, data), device="cpu")
    assert not hasattr(model.query_tower.embedding.embedding.weight, "_tt_deferred")
    cfg = _config(ref_pkg, data)
    cfg["hip"] = {"table_update": "backward"}
    model, _, optimizer, _ = train.build_pipeline(cfg, device="cpu")
    assert type(optimizer) is torch.optim.AdamW
    w = model.query_tower.embedding.embedding.weight
    upd = w._tt_deferred.on_backward
    assert isinstance(upd, tt.optim.BackwardTableUpdate) and upd.optimizer is optimizer and upd.weight is w
    assert getattr(optimizer, "_tt_dense_update", None) is None
    cfg["hip"] = {"table_update": "backward", "dense_update": "backward"}
    model, _, optimizer, _ = train.build_pipeline(cfg, device="cpu")
    dense = optimizer._tt_dense_update
    assert isinstance(dense, tt.optim.BackwardDenseUpdate) and dense.optimizer is optimizer
    assert {id(p) for p in dense.params} == {id(p) for p in model.parameters()} - {
        id(model.query_tower.embedding.embedding.weight)}
    cfg["hip"] = {"table_update": "sideways"}
    with pytest.raises(ValueError, match="table_update"):
        train.build_pipeline(cfg, device="cpu")
    cfg["hip"] = {"dense_update": "sideways"}
    with pytest.raises(ValueError, match="dense_update"):
        train.build_pipeline(cfg, device="cpu")


def test_backward_table_update_refuses_what_it_does_not_implement():
    import twotower_amd as tt

    emb = tt.embeddings.build("lookup", vocab_size=20, embedding_dim=8)
    model = tt.build_two_tower("mean", emb, hidden_dim=8, tied_weights=True)
    with pytest.raises(TypeError):
        tt.optim.fuse_table_update(torch.optim.SGD(model.parameters(), lr=0.1), model)
    with pytest.raises(ValueError, match="amsgrad"):
        tt.optim.fuse_table_update(torch.optim.AdamW(model.parameters(), amsgrad=True), model)
    ups = tt.optim.fuse_table_update(torch.optim.AdamW(model.parameters()), [model, emb])
    assert len(ups) == 1  # one shared table, attached once
    with pytest.raises(ValueError, match="already owned"):
        tt.optim.fuse_table_update(torch.optim.AdamW(model.parameters()), model)
