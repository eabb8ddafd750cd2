"""Multi-rank exchange path (directory sharded by ring owner, all-to-all-v) on
CPU with gloo, world sizes 2 and 3, launched like bench.py is for N > 1."""
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_exchange_gloo(world):
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "_gloo_worker.py")]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    for r in range(world):
        assert f"OK rank {r}/{world}" in out, out[-4000:]


@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_fanout_gloo(world):
    """The partitioned fan-out cascade's host logic (partition_graph_np / partition_graph_torch, the
    rank-local seed selection, per-hop exchange by owner rank) over gloo equals the replicated-graph
    oracle cascade (tests/_gloo_fanout_worker.py)."""
    env = dict(os.environ, OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "_gloo_fanout_worker.py")]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    out = p.stdout + p.stderr
    assert p.returncode == 0, out[-4000:]
    for r in range(world):
        assert f"OK rank {r}/{world} partitioned fan-out" in out, out[-4000:]
