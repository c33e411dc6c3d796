# Capture-time stand-in for the absent third-party ``yacs`` package (pinned 0.1.8 by
# the reference's requirements.txt).  Re-exports the restatement of its published
# CfgNode behaviour.  Used ONLY by tests/golden/make_golden.py in the build container.
from factmx.configs.cfgnode import CfgNode  # noqa: F401
