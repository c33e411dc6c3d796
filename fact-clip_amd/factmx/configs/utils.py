"""Config helpers with the reference's call surface.

* ``setup_cfg(cfg_file, set_cfgs)``  - fact_clip/configs/utils.py:172-216
* ``update_from(cfg, ref, inplace)`` - fact_clip/configs/utils.py:219-231
* ``int2float_check(x, tgt)``       - fact_clip/configs/utils.py:127-134
"""
import os

from .cfgnode import CfgNode
from .default import get_cfg_defaults


def int2float_check(x, tgt):
    """'--set lr 1' must become 1.0 when the default is a float."""
    if isinstance(tgt, float) and "." not in x:
        try:
            int(x)
            x = x + ".0"
        except ValueError:
            pass
    return x


def _lookup(node, dotted):
    for k in dotted.split("."):
        node = node[k]
    return node


def setup_cfg(cfg_file=(), set_cfgs=None, default: CfgNode = None, logdir="log/") -> CfgNode:
    cfg = get_cfg_defaults() if default is None else default.clone()
    overrides = []
    pairs = list(set_cfgs) if set_cfgs else []
    for k, v in zip(pairs[0::2], pairs[1::2]):
        for key in (k if isinstance(k, list) else [k]):
            overrides += [key, int2float_check(v, _lookup(cfg, key))]
    for f in cfg_file:
        cfg.merge_from_file(f)
    if overrides:
        cfg.merge_from_list(overrides)
    cfg.aux.cfg_file = list(cfg_file)
    cfg.aux.set_cfgs = set_cfgs
    names = [".".join(os.path.basename(f).split(".")[:-1]) for f in cfg_file]
    if len(cfg.aux.mark) > 0:
        names.append(cfg.aux.mark)
    cfg.aux.exp = "-".join(names) if names else "default"
    base = logdir if not cfg.aux.debug else "log_test/"
    cfg.aux.logdir = os.path.join(base, cfg.dataset, cfg.split, cfg.aux.exp, str(cfg.aux.runid)).replace("-", "_")
    return cfg


def update_from(cfg: CfgNode, ref: CfgNode, inplace=False) -> CfgNode:
    """Fill every None key of ``cfg`` from ``ref`` (block-config inheritance)."""
    if not inplace:
        cfg = cfg.clone()
    cfg.defrost()
    for k in cfg:
        if k in ref and cfg[k] is None and ref[k] is not None:
            cfg[k] = ref[k]
    return cfg
