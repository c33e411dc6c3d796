"""Capture config-layer golden vectors from the reference (build container only).

Run:  python tests/golden/make_cfg_golden.py   -> tests/golden/configs.json
For a few of the reference's yaml configs and ``--set`` lists, stores the
yaml's parsed contents (input data), the ``set_cfgs`` list, and the reference
``setup_cfg`` result (expected output, incl. the generated experiment name and
log dir).  The reference's ``yacs`` dependency is absent; ``_yacs_shim`` stands
in for it (see make_golden.py).
"""
import json
import os
import sys

import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(ROOT, "fact-clip_amd"))
sys.path.insert(0, os.path.join(HERE, "_yacs_shim"))
sys.path.insert(0, REF)

from fact_clip.configs import default as ref_default  # noqa: E402
from fact_clip.configs import utils as ref_utils  # noqa: E402

CASES = [
    ("havid_view0_lh_pt_holdout.yaml", ["FACT.ntoken", "32"]),
    ("havid_view0_lh_pt_holdout.yaml", None),
    ("breakfast.yaml", ["Bi.hid_dim", "256", "lr", "1", "aux.mark", "x1", "FACT.cmr", "0.2"]),
    ("gtea.yaml", ["Loss.match", "o2m", "FACT.trans", "True"]),
    ("havid_view1_rh_pt_holdout.yaml", [["Bi.dropout", "Bu.dropout"], "0.1"]),
]


def to_plain(node):
    if isinstance(node, dict):
        return {k: to_plain(v) for k, v in node.items()}
    if isinstance(node, tuple):
        return list(node)
    return node


def main():
    out = {"defaults": to_plain(ref_default.get_cfg_defaults()), "cases": []}
    for fname, sets in CASES:
        path = os.path.join(REF, "fact_clip", "configs", fname)
        with open(path) as f:
            ydata = yaml.safe_load(f)
        cfg = ref_utils.setup_cfg([path], sets)
        exp = to_plain(cfg)
        exp["aux"]["cfg_file"] = None   # absolute path of the capture machine; not compared
        out["cases"].append({"file": fname, "yaml": ydata, "set_cfgs": sets, "expected": exp})
    with open(os.path.join(HERE, "configs.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=False)
    print("wrote", len(out["cases"]), "cases")


if __name__ == "__main__":
    main()
