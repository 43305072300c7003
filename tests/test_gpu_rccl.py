"""The multi-GPU data path (fate_amd.dist: all-gather of ciphertext shards, compaction of
padded shards, the cross-rank histogram fold) on the real collective backend: RCCL
(torch.distributed "nccl"), world_size 1 on the box's GPU.  Runs in a fresh child process
(tests/rccl_child.py) so the process group is initialised before any other GPU work, as in a
bench.py rank.  Reference decomposition: python/fate/arch/tensor/distributed/_tensor.py:365-443."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.gpu
def test_rccl_gather_and_cross_rank_fold():
    r = subprocess.run([sys.executable, os.path.join(HERE, "rccl_child.py")], capture_output=True, text=True,
                       timeout=300, env=dict(os.environ))
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, f"no result line (rc {r.returncode}): {r.stderr[-2000:]}"
    res = json.loads(lines[-1])
    print(res)
    assert res["backend"] == "nccl"
    assert res["gather"] and res["compact"] and res["fold"], res
    assert r.returncode == 0
