"""Default config tree.

Same key names and default values as the reference's yacs defaults
(fact_clip/configs/default.py:3-148) so every reference yaml and ``--set``
override is a drop-in.  Declared here as one nested literal.
"""
from .cfgnode import CfgNode

_BLOCK_INHERIT = dict(hid_dim=None, dropout=None, a="sa", a_nhead=None, a_ffdim=None, a_layers=1,
                      a_dim=None, f=None, f_layers=5, f_ln=None, f_dim=None, f_ngp=None)

_DEFAULTS = {
    "aux": dict(gpu=1, mark="", runid=0, debug=False, wandb_project="FACT", wandb_user="",
                wandb_offline=False, resume="max", eval_every=1000, print_every=200),
    "dataset": "breakfast", "split": "split1", "sr": 1, "eval_bg": False,
    "feature_path": None, "groundTruth_path": None, "split_path": None, "map_fname": None,
    "feature_transpose": False, "bg_class": None, "average_transcript_len": 0.0,
    "holdout_mode": False, "holdout_classes": [],
    "use_clip": False,
    "batch_size": 4, "optimizer": "SGD", "epoch": 2, "lr": 0.1, "lr_decay": -1,
    "momentum": 0.009, "weight_decay": 0.0, "clip_grad_norm": 10.0,
    "FACT": dict(ntoken=30, block="iuUU", trans=False, fpos=True, cmr=0.3, mwt=0.1),
    "Bi": dict(hid_dim=512, dropout=0.5, a="sca", a_nhead=8, a_ffdim=2048, a_layers=6, a_dim=512,
               f="cnn", f_layers=10, f_ln=True, f_dim=512, f_ngp=4),
    "Bu": dict(_BLOCK_INHERIT),
    "BU": dict(_BLOCK_INHERIT, s_layers=1),
    "Loss": dict(pc=1.0, a2fc=1.0, match="o2o", bgw=1.0, nullw=-1.0, sw=0.0),
    "TM": dict(use=False, t=30, p=0.05, m=5, inplace=True),
    "CLIP": dict(model_name="openai/clip-vit-base-patch32", text_trainable=True, temp=0.07,
                 precompute_text=True, use_prompt=True, text_emb_path=None,
                 contrastive_weight=0.5, fact_loss_weight=0.5,
                 projection_hidden_dim=512, projection_dropout=0.1),
}

_C = CfgNode(_DEFAULTS)


def get_cfg_defaults():
    return _C.clone()
