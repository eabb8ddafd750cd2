"""The two-level bucketing (gd_msd.h, GD_MSD): a stable MSD pass into ranges of 1,024 activations,
then one workgroup per range sorting it in LDS and writing its bucket starts.  Its permutation and
offsets must equal the stable partition of the oracle (o.bucket_stable: the per-activation FIFO,
IncomingMessageAgent.cs:92-190, ActivationData.cs:566-606) and the LSD path's, for every shape the
path takes: range edges, the unrouted bucket n_act, empty ranges, ranges staged in LDS and ranges
over the staging capacity (hot activations: chunks stored straight to global memory), ranges either
side of that capacity in one launch, the largest n_act the MSD digit takes, and through the fused
route + bucket and the receive path (which also asks for the inverse permutation)."""
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


# the forms of the second level: the message indices loaded in k_msd_local's rank sweep and the
# range-local keys as u16 records (the default); the same on u32 keys; the indices loaded with the
# keys; u16 positions staged with the indices gathered at write-out
FORMS = {"late": {"GD_MSD_G16": "0", "GD_MSD_EARLY": "0", "GD_MSD_K16": "1"},
         "late32": {"GD_MSD_G16": "0", "GD_MSD_EARLY": "0", "GD_MSD_K16": "0"},
         "early": {"GD_MSD_G16": "0", "GD_MSD_EARLY": "1", "GD_MSD_K16": "0"},
         "g16": {"GD_MSD_G16": "1", "GD_MSD_EARLY": "0", "GD_MSD_K16": "0"}}


def _engine(gd, msd, form="late"):
    env = dict(FORMS[form], GD_MSD=msd)
    os.environ.update(env)
    try:
        return gd.GrainDispatch(device=0, table_capacity=1 << 12)
    finally:
        for k in env:
            os.environ.pop(k, None)


SHAPES = [
    # (n, n_act, kind)
    (1 << 20, 1 << 20, "uniform"),
    (1 << 22, 1 << 20, "uniform"),
    (3_000_017, 4096, "uniform"),
    (1_500_001, 4097, "uniform"),
    (1 << 21, 1056 * 1024 - 1, "uniform"),                     # the largest n_act of the MSD digit
    (1 << 20, 43 * 1024 - 1, "uniform"),                       # ~24.4 K a range: either side of MSD_CAP
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


@pytest.mark.parametrize("form", list(FORMS))
@pytest.mark.parametrize("n,n_act,kind", SHAPES)
def test_msd_bucket_vs_oracle(gd, n, n_act, kind, form):
    acts = _acts(n, n_act, kind, n + n_act)
    e2, e0 = _engine(gd, "2", form), _engine(gd, "0")
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


def test_msd_receive_with_limits(gd):
    """The receive path with overload limits asks the bucketing for the inverse permutation too
    (each message's place in its context's FIFO, IncomingMessageAgent.cs:142 CheckOverloaded):
    with the two-level form forced, statuses, contexts, permutation and offsets equal the oracle's."""
    import torch
    from test_gpu_receive import _world
    import receive as rv
    rng, keys, ctxs, flags, tg, ta, direction = _world(23, 1 << 18, 16, 1 << 21)
    n_ctx, n = len(keys), len(tg)
    e = _engine(gd, "2")
    e.actdir_add(keys, ctxs, flags)
    rc = rng.integers(0, 4, size=n_ctx).astype(np.uint32)
    dev = torch.device("cuda:0")
    d_tg = torch.from_numpy(tg.view(np.int64)).to(dev)
    d_ta = torch.from_numpy(ta.view(np.int64)).to(dev)
    d_dir = torch.from_numpy(direction).to(dev)
    d_rc = torch.from_numpy(rc.view(np.int32)).to(dev)
    ctx = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    perm = torch.empty(n, dtype=torch.int32, device=dev)
    off = torch.empty(n_ctx + 3, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    e.receive_device(d_tg.data_ptr(), d_ta.data_ptr(), d_dir.data_ptr(), n, n_ctx, ctx.data_ptr(), st.data_ptr(),
                     perm.data_ptr(), off.data_ptr(), d_rc.data_ptr(), 2, 1)
    e.synchronize()
    w = rv.receive_batch_np(tg, ta, direction, keys, ctxs, flags, n_ctx, rc, 2, 1)
    np.testing.assert_array_equal(st.cpu().numpy(), w[0])
    np.testing.assert_array_equal(ctx.cpu().numpy().view(np.uint32), w[1])
    np.testing.assert_array_equal(perm.cpu().numpy().view(np.uint32), w[2])
    np.testing.assert_array_equal(off.cpu().numpy().view(np.uint32), w[3])
    e.close()


def test_msd_measured_choice_per_shape(gd):
    """The measured choice is kept per batch size and per messages-a-range class: one handle
    alternating 2^21 messages over 2^20 activations (ranges staged in LDS) and over 10,000 (ranges
    far over the staging capacity) stays bit-exact on every launch, through both forms' timing."""
    e = _engine(gd, "1")
    shapes = [(_acts(1 << 21, 1 << 20, "uniform", 5), 1 << 20), (_acts(1 << 21, 10000, "uniform", 6), 10000)]
    want = [o.bucket_stable(a, na) for a, na in shapes]
    for i in range(10):
        a, na = shapes[i % 2]
        p, off = e.bucket(a, na)
        np.testing.assert_array_equal(p, want[i % 2][0])
        np.testing.assert_array_equal(off, want[i % 2][1])
    e.close()
