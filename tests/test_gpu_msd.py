"""The two-level bucketing (GD_OPT_BUCKET): ranges of 1,024 activations, each sorted stably in LDS.

One-pass form (gd_msd.h, n_act < 1,081,344): one MSD pass into the ranges, one workgroup a range.
Three-pass form (gd_msd2.h, n_act up to 2^28): two MSD passes (the second segmented, its positions
from one flat scan), then the ranges in three work lists -- thin ranges one wave each, staged ranges
one workgroup each, hot ranges in chunks over several workgroups.

The permutation and offsets must equal the stable partition of the oracle (o.bucket_stable: the
per-activation FIFO, IncomingMessageAgent.cs:92-190, ActivationData.cs:566-606) and the LSD path's,
for every shape the forms take: range edges, the unrouted bucket n_act, empty ranges, ranges either
side of each class boundary (the thin-range threshold, the staging capacity 24,576, whole numbers of
16,384-message chunks), Zipf-hot ranges, the largest n_act of each form, and through the fused route +
bucket and the receive path (which also asks for the inverse permutation)."""
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


def _engine(gd, bucket, **opts):
    """GD_OPT_BUCKET: 0 the LSD passes, 1 measured, 2 the two-level form wherever it applies."""
    return gd.GrainDispatch(device=0, table_capacity=1 << 12, options=dict(opts, bucket=int(bucket)))


ONE_PASS = [
    # (n, n_act, kind)
    (1 << 20, 1 << 20, "uniform"),
    (1 << 22, 1 << 20, "uniform"),
    (3_000_017, 4096, "uniform"),
    (1_500_001, 4097, "uniform"),
    (1 << 21, 1056 * 1024 - 1, "uniform"),                     # the largest n_act of the one-pass form
    (1 << 20, 43 * 1024 - 1, "uniform"),                       # ~24.4 K a range: either side of MSD_CAP
    (1 << 21, 1000, "uniform"),
    (1 << 21, 300_000, "unrouted"),
    (1 << 21, 1 << 20, "hot"),
    (1 << 22, 1 << 16, "sparse"),
]

THREE_PASS = [
    (1 << 20, 1056 * 1024, "uniform"),                         # the smallest n_act of the three-pass form
    (1 << 21, 1 << 21, "uniform"),                             # ~1,024 a range: thin / staged boundary
    (1 << 22, 1 << 21, "zipf"),                                # hot ranges in chunks
    (1 << 22, 1 << 21, "hot"),                                 # one activation with 70 % of the batch
    (1 << 22, 10_000_000, "zipf"),                             # BASELINE cfg 4's n_act
    (1 << 22, 100_000_000, "zipf"),                            # BASELINE cfg 3's n_act
    (1 << 21, 100_000_000, "uniform"),                         # ~21 messages a range
    (3_000_017, 5_000_000, "unrouted"),
    (1 << 21, 1 << 21, "edges"),                               # ranges of exactly 24,576 / 24,577 / 32,768 ...
    (1 << 20, (1 << 27) + 5, "uniform"),                       # 18-bit ranges: 9 + 9 digit bits
]


def _acts(n, n_act, kind, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, n_act, size=n, dtype=np.int64)
    if kind == "unrouted":
        a[rng.random(n) < 0.2] = 0xFFFFFFFF                     # GD_NO_ACTIVATION: the trailing bucket
        a[rng.random(n) < 0.05] = n_act + rng.integers(0, 5, size=n)[0]
    elif kind == "hot":
        a[rng.random(n) < 0.7] = 4095                           # one activation over many chunks
        a[rng.random(n) < 0.1] = 4096 * 7 + 3
    elif kind == "sparse":
        a = rng.choice(np.arange(0, n_act, 4099), size=n)       # most ranges empty or thin
    elif kind == "zipf":
        a = (rng.zipf(1.1, size=n) - 1) % n_act                 # Zipf(1.1): low activations hot
    elif kind == "edges":
        # whole ranges of chosen sizes around the class boundaries, the rest thin
        sizes = {5: 24576, 7: 24577, 9: 32768, 11: 32769, 13: 16384, 17: 1024, 19: 1025, 23: 49153}
        parts = [rng.integers(b * 1024, b * 1024 + 1024, size=s) for b, s in sizes.items()]
        rest = n - sum(sizes.values())
        r = rng.integers(0, n_act, size=rest)
        r = r[~np.isin(r >> 10, list(sizes))]
        a = np.concatenate(parts + [r])
        rng.shuffle(a)
    return a.astype(np.uint32)


def _check(gd, acts, n_act, **opts):
    e2, e0 = _engine(gd, 2, **opts), _engine(gd, 0)
    p2, off2 = e2.bucket(acts, n_act)
    p0, off0 = e0.bucket(acts, n_act)
    wp, wo = o.bucket_stable(acts, n_act)
    np.testing.assert_array_equal(p2, wp)
    np.testing.assert_array_equal(off2, wo)
    np.testing.assert_array_equal(p0, wp)
    np.testing.assert_array_equal(off0, wo)
    return e2, e0


@pytest.mark.parametrize("n,n_act,kind", ONE_PASS)
def test_msd_one_pass_vs_oracle(gd, n, n_act, kind):
    e2, e0 = _check(gd, _acts(n, n_act, kind, n + n_act), n_act)
    e2.close()
    e0.close()


@pytest.mark.parametrize("n,n_act,kind", THREE_PASS)
def test_msd_three_pass_vs_oracle(gd, n, n_act, kind):
    e2, e0 = _check(gd, _acts(n, n_act, kind, n + n_act + 3), n_act)
    e2.close()
    e0.close()


@pytest.mark.parametrize("n,n_act,kind", [ONE_PASS[0], ONE_PASS[4], ONE_PASS[8], THREE_PASS[1], THREE_PASS[2],
                                           THREE_PASS[3], THREE_PASS[5], THREE_PASS[8]])
def test_msd_ballot_ranks_vs_oracle(gd, n, n_act, kind):
    """Every bucketing form with its ranks by ballots (GD_CFG_NO_LANE_ORDER: the library's path on a
    device whose LDS atomics are not served in lane order) -- stable by construction -- equals the
    oracle: the one-pass and three-pass forms (thin, mid, staged and chunked ranges, the hot-key
    register path) and the LSD passes."""
    acts = _acts(n, n_act, kind, n + n_act + 11)
    wp, wo = o.bucket_stable(acts, n_act)
    for bucket in (2, 0):
        e = gd.GrainDispatch(device=0, table_capacity=1 << 12, options={"bucket": bucket}, no_lane_order=True)
        assert e.get_option("stable_rank") == 0
        p, off = e.bucket(acts, n_act)
        np.testing.assert_array_equal(p, wp, err_msg=f"bucket {bucket}")
        np.testing.assert_array_equal(off, wo, err_msg=f"bucket {bucket}")
        e.close()


@pytest.mark.parametrize("persist", [0, 1, 3])
@pytest.mark.parametrize("n,n_act,kind", [ONE_PASS[1], ONE_PASS[2], ONE_PASS[7], ONE_PASS[8]])
def test_msd_persistent_scatter_vs_oracle(gd, persist, n, n_act, kind):
    """GD_OPT_B2_PERSIST: the one-pass form's MSD scatter one workgroup a tile (0) or on k persistent
    workgroups a CU, each looping over its XCD's tiles with the next tile's loads under the current
    write-out (tiles past the grid, ragged last tiles, the unrouted bucket, hot digits); the default (2)
    runs in every other one-pass test; the result never changes."""
    e2, e0 = _check(gd, _acts(n, n_act, kind, n + n_act + 5), n_act, b2_persist=persist)
    e2.close()
    e0.close()


@pytest.mark.parametrize("small", [0, 300, 24576])
def test_msd_three_pass_class_threshold(gd, small):
    """The thin-range threshold moves ranges between the wave form and the workgroup form (0: every
    non-empty range staged; 24,576: every non-hot range a wave); the result never changes."""
    acts = _acts(1 << 21, 3 << 20, "zipf", 77)
    e2, e0 = _check(gd, acts, 3 << 20, l2_small=small)
    e2.close()
    e0.close()


@pytest.mark.parametrize("mid", [0, 2000, 8192])
def test_msd_three_pass_mid_class(gd, mid):
    """The mid-range class (512-thread sorts, GD_OPT_L2_MID) takes staged ranges up to `mid` messages,
    the 1,024-thread sort the rest (0: none mid); Zipf ranges from a few to 24K+ messages cover every
    class at each setting; the result never changes."""
    acts = _acts(1 << 22, 3 << 20, "zipf", 91)
    e2, e0 = _check(gd, acts, 3 << 20, l2_mid=mid)
    e2.close()
    e0.close()


@pytest.mark.parametrize("staged,small", [(2048, 1024), (0, 1024), (0, 0), (1100, 300)])
def test_msd_three_pass_small_staged_threshold(gd, staged, small):
    """GD_OPT_L2_STAGED below the staging capacity: every range over max(l2_small, l2_staged) messages
    is chunked (k_l2_classify), far more chunked ranges than the default's n / 24,577 -- the chunk
    buffers are sized from that threshold (msd3_bucket), and the result never changes.  Uniform
    ~2K-message ranges: most ranges exceed 2,048 / 1,024 / 0."""
    acts = _acts(1 << 22, 2 << 20, "uniform", 55)
    e2, e0 = _check(gd, acts, 2 << 20, l2_staged=staged, l2_small=small)
    e2.close()
    e0.close()
    acts = _acts(1 << 21, 3 << 20, "zipf", 56)
    e2, e0 = _check(gd, acts, 3 << 20, l2_staged=staged, l2_small=small)
    e2.close()
    e0.close()


def test_msd_three_pass_kernels(gd):
    """The three-pass form runs its own kernels (not the LSD passes) when forced."""
    acts = _acts(1 << 21, 5_000_000, "zipf", 9)
    e = _engine(gd, "2")
    e.set_kernel_timing(True)
    p, off = e.bucket(acts, 5_000_000)
    names = set(e.kernel_times())
    assert {"k_seg_hist", "k_seg_scatter", "k_l2_classify", "k_l2_small", "k_l2_chunk_scatter"} <= names, names
    assert "k_starts_rangescan" not in names
    wp, wo = o.bucket_stable(acts, 5_000_000)
    np.testing.assert_array_equal(p, wp)
    np.testing.assert_array_equal(off, wo)
    e.close()


def test_stage_timing_brackets_the_whole_bucketing(gd):
    """gd_set_kernel_timing 2: one event pair a bucketing ("stage:bucket"), no per-launch events; the
    stage takes no longer than the per-launch sum (which pays an event pair a kernel)."""
    acts = _acts(1 << 21, 5_000_000, "zipf", 19)
    e = _engine(gd, "2")
    e.bucket(acts, 5_000_000)                                    # scratch allocated outside the timing
    e.set_kernel_timing(2)
    e.kernel_times_reset()
    for _ in range(3):
        e.bucket(acts, 5_000_000)
    t = {k: v for k, v in e.kernel_times().items() if v[0]}
    assert set(t) == {"stage:bucket"} and t["stage:bucket"][0] == 3, t
    e.set_kernel_timing(True)
    e.kernel_times_reset()
    for _ in range(3):
        e.bucket(acts, 5_000_000)
    k = {n: v for n, v in e.kernel_times().items() if v[0]}
    assert "stage:bucket" not in k and "k_seg_scatter" in k
    assert t["stage:bucket"][1] <= 1.05 * sum(v[1] for v in k.values())
    e.close()


def test_msd_measured_choice_and_fused_route(gd):
    """GD_OPT_BUCKET 1 (the default): the first launches of a batch size alternate the two forms; every
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


@pytest.mark.parametrize("n_ctx", [1 << 18, 1_200_000])
def test_msd_receive_with_limits(gd, n_ctx):
    """The receive path with overload limits asks the bucketing for the inverse permutation too
    (each message's place in its context's FIFO, IncomingMessageAgent.cs:142 CheckOverloaded):
    with the two-level form forced (one-pass at 2^18 contexts, three-pass at 1.2M), statuses,
    contexts, permutation and offsets equal the oracle's."""
    import torch
    from test_gpu_receive import _world
    import receive as rv
    rng, keys, ctxs, flags, tg, ta, direction = _world(23, n_ctx, 16, 1 << 21)
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
    alternating 2^21 messages over 2^20 activations (ranges staged in LDS), over 10,000 (ranges far
    over the staging capacity) and over 3M (the three-pass form) stays bit-exact on every launch,
    through every form's timing."""
    e = _engine(gd, "1")
    shapes = [(_acts(1 << 21, 1 << 20, "uniform", 5), 1 << 20), (_acts(1 << 21, 10000, "uniform", 6), 10000),
              (_acts(1 << 21, 3_000_000, "zipf", 7), 3_000_000)]
    want = [o.bucket_stable(a, na) for a, na in shapes]
    for i in range(15):
        a, na = shapes[i % 3]
        p, off = e.bucket(a, na)
        np.testing.assert_array_equal(p, want[i % 3][0])
        np.testing.assert_array_equal(off, want[i % 3][1])
    e.close()
