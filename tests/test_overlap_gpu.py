"""Multi-GPU overlap evidence on one GPU: in the SC25 EGNN-866 multibranch step (bf16, the
captured configuration) the first gradient bucket's all-reduce must be enqueued while at
least a quarter of the backward kernels are still to come (tools/overlap_check.py, 1-rank
RCCL, HYDRA_GRADSYNC_FORCE=1), i.e. bucket collectives overlap the rest of backward instead
of all landing after the last backward kernel."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_first_bucket_allreduce_overlaps_backward():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "overlap_check.py"), "--config", "multibranch_egnn",
                        "--precision", "bf16"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    print(r.stdout[-3000:])
    print(r.stderr[-3000:])
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["allreduces"] >= 2 and res["backward_kernel_launches"] > 0, res
    assert res["fraction_after_first"] >= 0.25, res
