"""GPU parity of the two-pass wide-digit bucketing (gd_bucket2.h, GD_BUCKET2=1: a measured
alternative to the three 7-bit passes) against the oracle's stable partition
(ActivationData.cs:566-606 FIFO per activation, WorkItemGroup.cs:174-201).  Bit-exact perm and
offsets on uniform, Zipf-skewed and unrouted keys, ragged tile counts, and the smallest n_act the
path takes; and through the receive path's inverse permutation (CheckOverloaded)."""
import os

import numpy as np
import pytest

import oracle as o

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gd():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from orleans_amd import graindispatch as g
    return g


def _engine(gd):
    os.environ["GD_BUCKET2"] = "1"
    try:
        return gd.GrainDispatch(device=0, table_capacity=1024)
    finally:
        del os.environ["GD_BUCKET2"]


@pytest.mark.parametrize("n,n_act,dist", [(1 << 21, 1 << 20, "uniform"), ((1 << 20) + 12345, 1 << 20, "zipf"),
                                          (1 << 21, 70000, "uniform"), (3_000_001, 1_081_343, "unrouted")])
def test_bucket2_vs_oracle(gd, n, n_act, dist):
    rng = np.random.default_rng(n ^ n_act)
    if dist == "zipf":
        acts = np.minimum(rng.zipf(1.1, size=n) - 1, n_act - 1).astype(np.uint32)
    else:
        acts = rng.integers(0, n_act, size=n).astype(np.uint32)
    if dist == "unrouted":
        acts[rng.random(n) < 0.05] = 0xFFFFFFFF                  # unrouted: the trailing bucket
        acts[:7] = n_act
    e = _engine(gd)
    perm, off = e.bucket(acts, n_act)
    wp, wo = o.bucket_stable(acts, n_act)
    np.testing.assert_array_equal(perm, wp)
    np.testing.assert_array_equal(off, wo)
    e.close()
