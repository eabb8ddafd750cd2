"""The two-level bucketing (gd_msd.h, GD_MSD): a stable MSD pass into ranges of 4,096 activations,
then one workgroup per range sorting it in LDS and writing its bucket starts.  Its permutation and
offsets must equal the stable partition of the oracle (o.bucket_stable: the per-activation FIFO,
IncomingMessageAgent.cs:92-190, ActivationData.cs:566-606) and the LSD path's, for every shape the
path takes: range edges, the unrouted bucket n_act, empty ranges, ranges over one u16 chunk (hot
activations), and through the fused route + bucket and the receive path (which also asks for the
inverse permutation)."""
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


def _engine(gd, msd):
    os.environ["GD_MSD"] = msd
    try:
        return gd.GrainDispatch(device=0, table_capacity=1 << 12)
    finally:
        os.environ.pop("GD_MSD", None)


SHAPES = [
    # (n, n_act, kind)
    (1 << 20, 1 << 20, "uniform"),
    (1 << 22, 1 << 20, "uniform"),
    (3_000_017, 4096, "uniform"),
    (1_500_001, 4097, "uniform"),
    (1 << 21, (1 << 21) - 1, "uniform"),
    (1 << 21, 1000, "uniform"),
    (1 << 21, 300_000, "unrouted"),
    (1 << 21, 1 << 20, "hot"),
    (1 << 22, 1 << 16, "sparse"),
]


def _acts(n, n_act, kind, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, n_act, size=n, dtype=np.int64)
    if kind == "unrouted":
        a[rng.random(n) < 0.2] = 0xFFFFFFFF                     # GD_NO_ACTIVATION: the trailing bucket
        a[rng.random(n) < 0.05] = n_act + rng.integers(0, 5, size=n)[0]
    elif kind == "hot":
        a[rng.random(n) < 0.7] = 4095                           # one activation over many u16 chunks
        a[rng.random(n) < 0.1] = 4096 * 7 + 3
    elif kind == "sparse":
        a = rng.choice(np.arange(0, n_act, 4099), size=n)       # most ranges empty or thin
    return a.astype(np.uint32)


@pytest.mark.parametrize("n,n_act,kind", SHAPES)
def test_msd_bucket_vs_oracle(gd, n, n_act, kind):
    acts = _acts(n, n_act, kind, n + n_act)
    e2, e0 = _engine(gd, "2"), _engine(gd, "0")
    p2, off2 = e2.bucket(acts, n_act)
    p0, off0 = e0.bucket(acts, n_act)
    np.testing.assert_array_equal(p2, p0)
    np.testing.assert_array_equal(off2, off0)
    wp, wo = o.bucket_stable(acts, n_act)
    np.testing.assert_array_equal(p2, wp)
    np.testing.assert_array_equal(off2, wo)
    e2.close()
    e0.close()


def test_msd_measured_choice_and_fused_route(gd):
    """GD_MSD=1 (the default): the first launches of a batch size alternate the two forms; every
    result along the way is the stable partition."""
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    tc = o.grain_type_code(o.PING_GRAIN_CLASS)
    G = 1 << 16
    reg = o.grain_keys(tc, np.arange(G))
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    e = _engine(gd, "1")
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    e.register(reg, np.arange(G), owner)
    rng = np.random.default_rng(3)
    keys = o.grain_keys(tc, rng.integers(0, G + 500, size=1 << 20))
    want = o.route_batch_np(keys, spec, o.DirectoryArrays(reg, np.arange(G), owner))
    wp, wo = o.bucket_stable(want[2], G)
    for _ in range(6):
        st, silo, act, perm, off = e.route_bucket(keys, G)
        np.testing.assert_array_equal(act, want[2])
        np.testing.assert_array_equal(perm, wp)
        np.testing.assert_array_equal(off, wo)
    e.close()
