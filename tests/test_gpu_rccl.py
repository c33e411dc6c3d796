"""The RCCL data-parallel path on the one leased MI355X (BASELINE configs[3] leg).

A world-size-1 ``nccl`` (RCCL) process group in a child process (tests/rccl_worker.py) runs the
real FACT_CLIP T=4096 lockstep step through factmx.dp.DataParallel with the per-block bucket
schedule forced on: every block's bucket is all-reduced (ReduceOp.AVG) by RCCL from the
backward hooks, from a collective stream ordered after the compute stream and the library's side
stream.  Over one rank AVG is the identity, so the reduced flat gradient must be BITWISE equal to
the plain step's (and the plain step is checked to be bitwise deterministic first).  Reference
semantics: blocks.py:913-915 (per-video loss mean).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_world1_bucket_schedule_bitwise(tmp_path):
    out = str(tmp_path)
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "rccl_worker.py"), "--out", out,
                        "--time-steps", "3"], env=env, timeout=300)
    assert p.returncode == 0, p.returncode
    r = np.load(os.path.join(out, "rccl.npz"))
    with open(os.path.join(out, "rccl.json")) as f:
        meta = json.load(f)
    assert meta["backend"] == "nccl"
    np.testing.assert_array_equal(r["plain1"], r["plain2"])          # the step is deterministic
    assert np.isfinite(r["forced"]).all()
    np.testing.assert_array_equal(r["forced"], r["plain1"])          # AVG over one rank == identity
    assert r["loss"][0] == r["loss"][1] == r["loss"][2]
    nblk = int(r["nblk"])
    # block buckets from the hooks, last block first, then block 0's action branch (-1) from the hook on
    # its frame-branch output; block 0's frame branch (its input is the data) at finish: <= 16 MB
    assert r["early"].tolist() == list(range(nblk - 1, 0, -1)) + [-1], r["early"]
    assert 0 < int(r["tail"]) <= 16 * 2 ** 20, int(r["tail"])
