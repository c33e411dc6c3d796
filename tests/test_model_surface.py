"""Drop-in surface of the product modules, checked on CPU (no kernels launched).

Construction order, parameter names and shapes must equal the reference's
``named_parameters()`` (captured into the golden fixtures' meta by
tests/golden/make_golden.py), so reference ``.net`` checkpoints load with
``load_state_dict`` unchanged (reference blocks.py:919-920).
"""
import pytest
import numpy as np
import torch

from helpers import cfg_from_meta, load_fixture, tiny_inputs, tiny_meta
from factmx.models.blocks import FACT, FACT_CLIP


def _build(name):
    fx = load_fixture(name)
    meta = tiny_meta(fx)
    cfg = cfg_from_meta(meta)
    _, _, text = tiny_inputs(meta)
    if meta["model"] == "FACT_CLIP":
        net = FACT_CLIP(cfg, meta["D"], meta["C"], torch.from_numpy(text).float())
    else:
        net = FACT(cfg, meta["D"], meta["C"])
    return net, meta


@pytest.mark.parametrize("name", ["tiny_clip", "tiny_clip_iid", "tiny_fact_m2"])
def test_parameter_names_order_and_shapes(name):
    net, meta = _build(name)
    got = [(n, list(p.shape)) for n, p in net.named_parameters()]
    exp = list(meta["param_shapes"].items())
    assert got == [(n, s) for n, s in exp]


@pytest.mark.parametrize("name", ["tiny_clip", "tiny_fact_m2"])
def test_buffers_match_reference(name):
    # reference: PositionalEncoding registers 'pe' (basic.py:103); FACT_CLIP registers
    # 'text_embeddings' when given (blocks.py:586)
    net, meta = _build(name)
    bufs = {n for n, _ in net.named_buffers()}
    exp = {"frame_pe.pe"} | ({"text_embeddings"} if meta["model"] == "FACT_CLIP" else set())
    assert bufs == exp


def test_state_dict_roundtrip():
    net, meta = _build("tiny_clip")
    sd = {k: v.clone() for k, v in net.state_dict().items()}
    for v in sd.values():
        v.add_(0.25)
    net2, _ = _build("tiny_clip")
    net2.load_state_dict(sd, strict=True)
    for k, v in net2.state_dict().items():
        assert torch.equal(v, sd[k]), k


def test_block_layout_follows_config():
    net, meta = _build("tiny_clip")
    kinds = [type(b).__name__ for b in net.block_list]
    assert kinds == ["InputBlock", "UpdateBlock", "UpdateBlockTDU", "UpdateBlockTDU"]  # FACT.block 'iuUU'
    assert net.action_query.shape == (meta["FACT"]["ntoken"], 1, meta["Bi"]["a_dim"])


def test_dropout_seed_follows_torch_manual_seed():
    # training dropout inside the fused kernels draws one seed per site from torch's CPU generator:
    # torch.manual_seed fixes the masks as it fixes nn.Dropout's
    from factmx import functional as fxf
    torch.manual_seed(3)
    a = [fxf.dropout_seed() for _ in range(3)]
    torch.manual_seed(3)
    b = [fxf.dropout_seed() for _ in range(3)]
    assert a == b and len(set(a)) == 3


def test_dropout_mask_keep_rate_host_restatement():
    from helpers import drop_mask
    keep = drop_mask(12345, np.arange(200000), 0.2)
    assert abs(keep.mean() - 0.8) < 4 * np.sqrt(0.16 / 200000)
    assert drop_mask(7, np.arange(1000), 0.0).all()
