"""CPU checks of bench.py's launcher contract (no GPU is touched): a world size that differs
from --gpus is an error before any device call, and `--gpus N` without a launcher re-runs the
same arguments as N torch.distributed.run ranks on 127.0.0.1 (--n passed as --elements)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_world_size_mismatch_is_an_error():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "--gpus 2 but the launcher started 1 rank(s)" in r.stderr


def test_rank_command_line():
    import bench
    cmd = bench.rank_command(4, 29511, ["--gpus", "4", "--n", "4096", "--steps=3", "--n=64", "--total", "100"])
    i = cmd.index("torch.distributed.run")
    assert cmd[i - 1] == "-m" and cmd[0] == sys.executable
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and "--master-port=29511" in cmd
    tail = cmd[cmd.index(os.path.abspath(bench.__file__)) + 1:]
    assert tail == ["--gpus", "4", "--elements", "4096", "--steps=3", "--elements=64", "--total", "100"]
