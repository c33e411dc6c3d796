"""Config helpers with the reference's call surface.

* ``setup_cfg(cfg_file, set_cfgs)``  - fact_clip/configs/utils.py:172-216
* ``update_from(cfg, ref, inplace)`` - fact_clip/configs/utils.py:219-231
* ``int2float_check(x, tgt)``       - fact_clip/configs/utils.py:127-134
* ``generate_expname`` / ``generate_diff_dict`` / ``diff2expname`` / ``cfg2flatdict``
  - fact_clip/configs/utils.py:5-125 (experiment name = config-file stems, then the
  non-aux keys that differ from default+files as ``Sec[key:val]``, then ``aux.mark``)
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


def cfg2flatdict(cfg: CfgNode, type_convert=True) -> dict:
    """{'Sec.key': value} over the whole tree (reference utils.py:27-40)."""
    out = {}

    def walk(node, prefix):
        for k, v in node.items():
            if isinstance(v, CfgNode):
                walk(v, prefix + k + ".")
            else:
                out[prefix + k] = v

    walk(cfg, "")
    if type_convert:
        out = {k: (v if type(v) in (int, float, bool, str) or type(v).__name__ == "Tensor" else str(v))
               for k, v in out.items()}
    return out


def generate_diff_dict(default: CfgNode, cfg: CfgNode, include_missing=False) -> dict:
    """Nested dict of the leaves of ``cfg`` that differ from ``default`` (utils.py:43-63)."""
    diff = {}
    for k, v in cfg.items():
        if k not in default:
            if not include_missing:
                continue
        if isinstance(v, CfgNode):
            sub = generate_diff_dict(default[k], v, include_missing=include_missing)
            if sub:
                diff[k] = sub
        elif v != default[k]:
            diff[k] = v
    return diff


def diff2expname(diff: dict, remove_leaf=False) -> str:
    """'Sec[key:val-key2:T]-key3:v' (bools abbreviated to T/F; aux and split skipped)."""
    parts = []
    for k, v in diff.items():
        if k.lower() in ("aux", "split"):
            continue
        if isinstance(v, dict):
            parts.append(f"{k}[{diff2expname(v)}]")
        elif not remove_leaf:
            parts.append(f"{k}:{str(v)[0] if isinstance(v, bool) else v}")
    return "-".join(parts)


_FILE_CACHE = {}


def generate_expname(cfg: CfgNode, cfg_file=None, default=None) -> str:
    cfg_file = cfg.aux.cfg_file if cfg_file is None else cfg_file
    ref = get_cfg_defaults() if default is None else default.clone()
    names = []
    for f in cfg_file:
        if f not in _FILE_CACHE:
            with open(f) as fp:
                _FILE_CACHE[f] = CfgNode.load_cfg(fp)
        ref.merge_from_other_cfg(_FILE_CACHE[f])
        names.append(".".join(os.path.basename(f).split(".")[:-1]))
    diff = {k[0].upper() + k[1:]: v for k, v in generate_diff_dict(ref, cfg).items()}
    tail = diff2expname(diff)
    if tail:
        names.append(tail)
    if len(cfg.aux.mark) > 0:
        names.append(cfg.aux.mark)
    return "-".join(names)


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
    cfg.aux.exp = generate_expname(cfg, default=default)
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
