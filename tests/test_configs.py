"""Config layer (factmx.configs) vs reference setup_cfg outputs (tests/golden/configs.json,
captured by tests/golden/make_cfg_golden.py from fact_clip/configs/{default,utils}.py)."""
import json
import os

import pytest
import yaml

from factmx.configs import CfgNode, get_cfg_defaults, setup_cfg, update_from
from factmx.configs.utils import generate_diff_dict, diff2expname

GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "configs.json")))


def plain(node):
    if isinstance(node, dict):
        return {k: plain(v) for k, v in node.items()}
    if isinstance(node, tuple):
        return list(node)
    return node


def test_defaults_identical():
    assert plain(get_cfg_defaults()) == GOLD["defaults"]


@pytest.mark.parametrize("case", GOLD["cases"], ids=lambda c: c["file"] + str(c["set_cfgs"]))
def test_setup_cfg_matches_reference(tmp_path, case):
    path = tmp_path / case["file"]
    path.write_text(yaml.safe_dump(case["yaml"]))
    cfg = setup_cfg([str(path)], case["set_cfgs"])
    got = plain(cfg)
    assert got["aux"]["cfg_file"] == [str(path)]
    got["aux"]["cfg_file"] = None
    assert got == case["expected"]


def test_type_rules():
    cfg = get_cfg_defaults()
    with pytest.raises(ValueError):
        cfg.merge_from_list(["Bi.hid_dim", "'abc'"])          # str into an int key
    with pytest.raises(KeyError):
        cfg.merge_from_list(["Bi.no_such_key", "1"])
    cfg.merge_from_list(["lr", "0.5"])
    assert cfg.lr == 0.5
    cfg.freeze()
    with pytest.raises(AttributeError):
        cfg.lr = 0.1
    c2 = cfg.clone()
    assert c2.is_frozen() and c2.lr == 0.5


def test_update_from_fills_none_only():
    cfg = get_cfg_defaults()
    bu = update_from(cfg.Bu, cfg.Bi)
    for k in cfg.Bu:
        if cfg.Bu[k] is None and k in cfg.Bi:
            assert bu[k] == cfg.Bi[k]
        else:
            assert bu[k] == cfg.Bu[k]
    assert isinstance(bu, CfgNode)


def test_expname_pieces():
    a = get_cfg_defaults()
    b = a.clone()
    b.Bi.hid_dim = 7
    b.FACT.trans = not a.FACT.trans
    d = generate_diff_dict(a, b)
    assert d == {"Bi": {"hid_dim": 7}, "FACT": {"trans": b.FACT.trans}}
    assert diff2expname({"Bi": d["Bi"], "aux": {"x": 1}, "split": "s"}) == "Bi[hid_dim:7]"
    assert diff2expname({"FACT": d["FACT"]}) == f"FACT[trans:{str(b.FACT.trans)[0]}]"
