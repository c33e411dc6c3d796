from .cfgnode import CfgNode
from .default import get_cfg_defaults
from .utils import setup_cfg, update_from, int2float_check

__all__ = ["CfgNode", "get_cfg_defaults", "setup_cfg", "update_from", "int2float_check"]
