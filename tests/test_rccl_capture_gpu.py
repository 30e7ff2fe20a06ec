"""The production multi-GPU gradient path on one GPU: a 1-rank RCCL (``nccl``) group with
the bucket all-reduces recorded into the captured training-step graph on the comm stream
(``parallel/ddp.py`` BucketedGradSync, forced with HYDRA_GRADSYNC_FORCE=1) must reproduce
the unsynced captured step bit for bit (``tools/gradsync_check.py``, run in a fresh child
process so the process group never leaks into other tests)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("mode", ["ddp", "taskpar"])
def test_captured_rccl_gradsync_one_rank(mode):
    """``taskpar``: MultiTaskModelMP in the captured step (encoder + branch-group syncs)."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    extra = ["--taskpar"] if mode == "taskpar" else []
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gradsync_check.py")] + extra, cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=300)
    print(r.stdout[-3000:])
    print(r.stderr[-3000:])
    assert r.returncode == 0 and "GRADSYNC_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]
