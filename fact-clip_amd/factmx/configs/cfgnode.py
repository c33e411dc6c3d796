"""yacs-compatible config node.

The reference builds its config on ``yacs==0.1.8`` (requirements.txt:7), which
is not installed in this image.  This module restates the published behaviour
of ``yacs.config.CfgNode`` that the FACT config surface relies on
(fact_clip/configs/default.py, utils.py): attribute access over a dict,
``clone``/``freeze``/``defrost``, ``merge_from_file`` (yaml, safe loader),
``merge_from_list`` (dotted keys, ``literal_eval`` values), ``merge_from_other_cfg``
and the type-coercion rules (None <-> valid type, list <-> tuple; anything else
must keep its type; unknown keys raise ``KeyError``).
"""
import copy
from ast import literal_eval

import yaml

_VALID = (tuple, list, str, int, float, bool, type(None))


class CfgNode(dict):
    IMMUTABLE = "__immutable__"

    def __init__(self, init_dict=None, key_list=None, new_allowed=False):
        init_dict = {} if init_dict is None else init_dict
        for k, v in list(init_dict.items()):
            if isinstance(v, dict) and not isinstance(v, CfgNode):
                init_dict[k] = CfgNode(v, new_allowed=new_allowed)
        super().__init__(init_dict)
        self.__dict__[CfgNode.IMMUTABLE] = False
        self.__dict__["__new_allowed__"] = new_allowed

    # attribute access ---------------------------------------------------
    def __getattr__(self, name):
        if name in self:
            return self[name]
        raise AttributeError(name)

    def __setattr__(self, name, value):
        if self.__dict__.get(CfgNode.IMMUTABLE, False):
            raise AttributeError(f"Attempted to set {name} to {value}, but CfgNode is immutable")
        self[name] = value

    def __str__(self):
        def _fmt(node, indent):
            lines = []
            for k in sorted(node):
                v = node[k]
                if isinstance(v, CfgNode):
                    lines.append(" " * indent + f"{k}:")
                    lines.append(_fmt(v, indent + 2))
                else:
                    lines.append(" " * indent + f"{k}: {v}")
            return "\n".join(lines)
        return _fmt(self, 0)

    def __repr__(self):
        return f"CfgNode({dict.__repr__(self)})"

    # mutability ---------------------------------------------------------
    def _set_immutable(self, flag):
        self.__dict__[CfgNode.IMMUTABLE] = flag
        for v in self.values():
            if isinstance(v, CfgNode):
                v._set_immutable(flag)

    def freeze(self):
        self._set_immutable(True)

    def defrost(self):
        self._set_immutable(False)

    def is_frozen(self):
        return self.__dict__[CfgNode.IMMUTABLE]

    def clone(self):
        return copy.deepcopy(self)

    def __deepcopy__(self, memo):
        node = CfgNode({k: copy.deepcopy(v, memo) for k, v in self.items()},
                       new_allowed=self.__dict__.get("__new_allowed__", False))
        node.__dict__[CfgNode.IMMUTABLE] = self.__dict__.get(CfgNode.IMMUTABLE, False)
        return node

    # merging --------------------------------------------------------------
    @classmethod
    def load_cfg(cls, cfg_file_obj_or_str):
        if isinstance(cfg_file_obj_or_str, str):
            data = yaml.safe_load(cfg_file_obj_or_str)
        else:
            data = yaml.safe_load(cfg_file_obj_or_str.read())
        return cls(data or {})

    def merge_from_file(self, cfg_filename):
        with open(cfg_filename, "r") as f:
            other = self.load_cfg(f)
        self.merge_from_other_cfg(other)

    def merge_from_other_cfg(self, cfg_other):
        _merge_a_into_b(cfg_other, self, self, [])

    def merge_from_list(self, cfg_list):
        if len(cfg_list) % 2 != 0:
            raise ValueError(f"Override list has odd length: {cfg_list}")
        root = self
        for full_key, v in zip(cfg_list[0::2], cfg_list[1::2]):
            keys = full_key.split(".")
            d = self
            for sub in keys[:-1]:
                if sub not in d:
                    raise KeyError(f"Non-existent key: {full_key}")
                d = d[sub]
            sub = keys[-1]
            if sub not in d:
                raise KeyError(f"Non-existent key: {full_key}")
            value = _decode(v)
            value = _coerce(value, d[sub], sub, full_key)
            d[sub] = value
        return root


def _decode(v):
    if isinstance(v, dict):
        return CfgNode(v)
    if not isinstance(v, str):
        return v
    try:
        return literal_eval(v)
    except (ValueError, SyntaxError):
        return v


def _coerce(replacement, original, key, full_key):
    rt, ot = type(replacement), type(original)
    if rt == ot:
        return replacement
    if (rt is type(None) and ot in _VALID) or (ot is type(None) and rt in _VALID):
        return replacement
    for a, b in ((tuple, list), (list, tuple)):
        if rt == a and ot == b:
            return b(replacement)
    raise ValueError(f"Type mismatch ({ot} vs. {rt}) with values ({original} vs. {replacement}) for config key: {full_key}")


def _merge_a_into_b(a, b, root, key_list):
    for k, v_ in a.items():
        full_key = ".".join(key_list + [k])
        v = copy.deepcopy(v_)
        v = _decode(v)
        if k in b:
            v = _coerce(v, b[k], k, full_key)
            if isinstance(v, CfgNode):
                _merge_a_into_b(v, b[k], root, key_list + [k])
            else:
                b[k] = v
        elif b.__dict__.get("__new_allowed__", False):
            b[k] = v
        else:
            raise KeyError(f"Non-existent config key: {full_key}")
