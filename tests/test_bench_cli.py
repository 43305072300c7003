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


def test_keyholder_credit_follows_the_draw(monkeypatch):
    """rooflines' key-holder credit (bench.enc_crt_mac32_per_elem) counts the modexps that run:
    with the (z_p, z_q) draw one |p|-bit exponent mod s^2 per half, else the split (keys above
    1024 bits: an extra |p|-bit exponent mod s) or one |n|-bit exponent mod s^2; and
    bench.kh_direct_z mirrors the library's switch (FPHE_KH_DIRECT_Z, gcd(q, p-1) =
    gcd(p, q-1) = 1)."""
    import bench
    for bits in (1024, 2048, 4096):
        d, r = bench.enc_crt_mac32_per_elem(bits, True), bench.enc_crt_mac32_per_elem(bits, False)
        assert 0 < d < r
    # 2048 bits: per half (1024 + 205 + 16) products over the 64-word p^2 against two such
    # exponents (mod p, then mod p^2): the direct draw saves the first step only
    rec = 4 * bench.mac32_per_mont(128)
    assert bench.enc_crt_mac32_per_elem(2048, True) == 2 * 1245 * bench.mac32_per_mont(64) + rec
    p, q = 1019, 1031  # q does not divide p - 1, p does not divide q - 1
    monkeypatch.delenv("FPHE_KH_DIRECT_Z", raising=False)
    assert bench.kh_direct_z(p, q)
    assert not bench.kh_direct_z(11, 23)  # 11 | 23 - 1
    monkeypatch.setenv("FPHE_KH_DIRECT_Z", "0")
    assert not bench.kh_direct_z(p, q)
