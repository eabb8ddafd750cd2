"""GPU parity at the BASELINE.json configurations that the other GPU tests do not reach.

* cfg 1 -- the Ping benchmark's shape (test/Benchmarks/Benchmarks/Ping/PingBenchmark.cs:15-35,
  BASELINE "1M IPingGrain calls over 10k grains, single in-process silo"): 1,048,576 calls over
  10,000 Ping grains on one silo (and on the 2-silo TestCluster default,
  src/Orleans.TestingHost/TestClusterBuilder.cs:22-36), every output compared with the oracle.
* cfg 3 at full size on one GPU -- 67,108,864 Zipf(1.1) messages over 100,000,000 grains
  (SURVEY 8 d): routes checked against the known directory, a 100k-message oracle sample, and the
  bucketing by size-independent properties (permutation, sorted, stable, offsets = counts).
* cfg 3's exchange at W = 8 (the node's GPU count) through the in-process transport
  (gd_comm_init_local): Zipf keys, owner-side arrival order, routes, buckets and returned routes
  against the oracle, then the bench's timed mode (GD_MULTI_KEYS_READY | GD_MULTI_NO_KEYS,
  pipelined device batches).
* The radix histogram variants (1, 4 and 8 tiles per workgroup) on ragged, unaligned inputs.
"""
import os

import numpy as np
import pytest

import oracle as o

pytestmark = pytest.mark.gpu

TC = o.grain_type_code(o.PING_GRAIN_CLASS)
TCD = o.type_code_data(o.CAT_GRAIN, TC)


@pytest.fixture(autouse=True)
def _region_order(monkeypatch, gd):
    """These tests expect the region-grouped arrival order (GD_OPT_REGION_PROBE = 1, the sender's option);
    test_route_multi_local_world_plain_order runs the other."""
    monkeypatch.setitem(gd.DEFAULT_OPTIONS, "region_probe", 1)


@pytest.fixture(scope="module")
def gd():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from orleans_amd import graindispatch as g
    return g


def _tuples(silos):
    return [(s.ip, s.port, s.gen) for s in silos]


# ----------------------------------------------------------------------------- cfg 1
@pytest.mark.parametrize("n_silos,mode", [(1, "D"), (2, "D"), (2, "V")])
def test_cfg1_ping_shape(gd, n_silos, mode):
    """1M Ping calls over 10k grains (one activation each, on the owner silo), route + bucket,
    compared in full with the oracle."""
    silos = o.bench_silos(n_silos)
    spec = o.ring_spec(silos, mode)
    G, N = 10_000, 1 << 20
    reg = o.grain_keys(TC, np.arange(G))
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    e = gd.GrainDispatch(device=0, table_capacity=2 * G)
    e.ring_set_silos(mode, _tuples(silos))
    e.register(reg, np.arange(G), owner)
    rng = np.random.default_rng(0x5EED0101)
    keys = o.grain_keys(TC, rng.integers(0, G, size=N))
    st, silo, act, perm, off = e.route_bucket(keys, G)
    want = o.route_batch_np(keys, spec, o.DirectoryArrays(reg, np.arange(G), owner))
    np.testing.assert_array_equal(st, want[0])
    np.testing.assert_array_equal(silo, want[1])
    np.testing.assert_array_equal(act, want[2])
    wp, wo = o.bucket_stable(want[2], G)
    np.testing.assert_array_equal(perm, wp)
    np.testing.assert_array_equal(off, wo)
    assert (st == o.ST_OK).all()
    e.close()


# ----------------------------------------------------------------------------- cfg 3, one GPU
def test_cfg3_full_size_one_gpu(gd):
    """67,108,864 Zipf(1.1) messages over 100,000,000 grains, route + bucket on one GPU.  The
    directory is built in HBM (gd_dir_register_device), act = grain index, silo = ring owner."""
    import torch
    from orleans_amd.workloads import grain_keys_torch, zipf_keys_torch
    dev = torch.device("cuda:0")
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    G, N = 100_000_000, 1 << 26
    e = gd.GrainDispatch(device=0, table_capacity=1 << 28)
    e.ring_set_silos("D", _tuples(silos))
    # a dedicated stream: torch's legacy default stream has handle 0, which gd_set_stream reads as
    # "the library's own (non-blocking) stream" -- torch's writes would then race the library
    stream = torch.cuda.Stream(dev)
    e.set_stream(stream.cuda_stream)
    ctx = torch.cuda.stream(stream)
    ctx.__enter__()
    owner = torch.empty(G, dtype=torch.int32, device=dev)
    chunk = 1 << 25
    for c0 in range(0, G, chunk):                    # the 100M registrations, in 32M chunks
        c1 = min(G, c0 + chunk)
        rk = grain_keys_torch(TCD, torch.arange(c0, c1, device=dev), dev)
        e.ring_owner_device(rk.data_ptr(), c1 - c0, owner[c0:c1].data_ptr())
        vals = torch.stack([torch.arange(c0, c1, device=dev, dtype=torch.int32), owner[c0:c1]], dim=1).contiguous()
        e.register_device(rk.data_ptr(), vals.data_ptr(), c1 - c0)
        del rk, vals
    assert e.stats()["table_live"] == G
    keys = zipf_keys_torch(TCD, G, N, 0x5EED0003, dev)
    silo = torch.empty(N, dtype=torch.int32, device=dev)
    act = torch.empty(N, dtype=torch.int32, device=dev)
    st = torch.empty(N, dtype=torch.uint8, device=dev)
    perm = torch.empty(N, dtype=torch.int32, device=dev)
    off = torch.empty(G + 2, dtype=torch.int32, device=dev)
    e.route_bucket_device(keys.data_ptr(), N, G, silo.data_ptr(), act.data_ptr(), st.data_ptr(), perm.data_ptr(),
                          off.data_ptr())
    torch.cuda.synchronize()
    k = keys[:, 1]
    assert bool((st == 0).all())
    assert bool((act.long() == k).all())
    assert bool((silo == owner[k]).all())
    # the ring owner on the GPU agrees with the oracle on a sample of the directory
    rng = np.random.default_rng(3)
    gs = rng.integers(0, G, size=200_000)
    rk = o.grain_keys(TC, gs)
    np.testing.assert_array_equal(owner[torch.from_numpy(gs).to(dev)].cpu().numpy().view(np.uint32),
                                  o.ring_owner_np(spec, o.jenkins_u64x3_np(rk[:, 2], rk[:, 0], rk[:, 1])))
    # 100k messages against the oracle (directory restricted to the sampled grains: exact for them)
    samp = torch.from_numpy(rng.choice(N, size=100_000, replace=False)).to(dev)
    sk = keys[samp].cpu().numpy().view(np.uint64)
    sg = sk[:, 1].astype(np.int64)
    sown = o.ring_owner_np(spec, o.jenkins_u64x3_np(sk[:, 2], sk[:, 0], sk[:, 1])).astype(np.uint32)
    want = o.route_batch_np(sk, spec, o.DirectoryArrays(sk, sg.astype(np.uint32), sown))
    np.testing.assert_array_equal(st[samp].cpu().numpy(), want[0])
    np.testing.assert_array_equal(silo[samp].cpu().numpy().view(np.uint32), want[1])
    np.testing.assert_array_equal(act[samp].cpu().numpy().view(np.uint32), want[2])
    # bucketing: a permutation, sorted by activation, stable, offsets = counts
    p = perm.long()
    seen = torch.zeros(N, dtype=torch.int32, device=dev)
    seen.index_add_(0, p, torch.ones(N, dtype=torch.int32, device=dev))
    assert bool((seen == 1).all())
    a_sorted = act[p].long()
    d = a_sorted[1:] - a_sorted[:-1]
    assert bool((d >= 0).all())
    assert bool(((p[1:] - p[:-1])[d == 0] > 0).all())
    counts = torch.bincount(act.long(), minlength=G + 1)
    offs = off.long()
    assert int(offs[0]) == 0 and int(offs[-1]) == N
    assert bool(((offs[1:] - offs[:-1]) == counts).all())
    # the hottest activation (rank 0) holds its Zipf share, in arrival order
    n0 = int(counts[0])
    assert n0 > N // 20
    assert bool((p[:n0] == torch.nonzero(k == 0).flatten()).all())
    ctx.__exit__(None, None, None)
    e.close()


# ----------------------------------------------------------------------------- cfg 3 exchange, W = 8
def _run_ranks(fns):
    import threading
    out, err = [None] * len(fns), [None] * len(fns)

    def body(r):
        try:
            out[r] = fns[r]()
        except BaseException as ex:           # noqa: BLE001 -- re-raised below
            err[r] = ex

    ts = [threading.Thread(target=body, args=(r,)) for r in range(len(fns))]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=110)
    for r, ex in enumerate(err):
        if ex is not None:
            raise AssertionError(f"rank {r}") from ex
    assert all(not t.is_alive() for t in ts), "a rank did not finish"
    return out


def test_cfg3_exchange_w8_zipf(gd):
    """cfg 3's sharded path at W = 8 ranks on one GPU: each rank owns the directory partitions of
    silo r (8 silos, rank = silo % 8), Zipf(1.1) batches; owner-side results and returned routes vs
    the oracle, then three pipelined batches in the bench's timed mode (keys ready, no key rebuild)
    checked by (sender, index), routes and buckets."""
    import torch
    from orleans_amd.sharded import _view
    from orleans_amd.workloads import zipf_ranks_np
    W, G = 8, 400_000
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    reg = o.grain_keys(TC, np.arange(G))
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    act = np.zeros(G, np.uint32)
    for r in range(W):                            # activation indices local to the owner rank
        act[own % W == r] = np.arange(int((own % W == r).sum()))
    n_act = [int((own % W == r).sum()) for r in range(W)]
    es = []
    for r in range(W):
        e = gd.GrainDispatch(device=0, table_capacity=1 << 18, my_silo=r)
        e.ring_set_silos("D", _tuples(silos))
        mine = own % W == r
        e.register(reg[mine], act[mine], own[mine])
        es.append(e)
    gd.GrainDispatch.comm_init_local(es)
    full = o.DirectoryArrays(reg, act, own)
    sizes = [60_000 + 7_919 * r for r in range(W)]
    batches = [o.grain_keys(TC, zipf_ranks_np(G, sizes[r], 0x5EED0003 + r)) for r in range(W)]

    def owner_side(bs, r):
        ks, ids, srcs = [], [], []
        for s, k in enumerate(bs):
            _, _, _, owner, _ = o.route_batch_np(k, spec, full, my_silo=s)
            sel = np.nonzero(owner % W == r)[0]
            sel = sel[o.region_order(k[sel])]     # arrival: (sender, table region, sender order)
            ks.append(k[sel]), ids.append(sel), srcs.append(np.full(len(sel), s))
        rk = np.concatenate(ks)
        stt, sl, a, _, _ = o.route_batch_np(rk, spec, full, my_silo=r)
        return rk, np.concatenate(ids).astype(np.uint32), np.concatenate(srcs).astype(np.uint32), stt, sl, a

    res = _run_ranks([lambda r=r: es[r].route_multi(batches[r], n_act[r], return_routes=True) for r in range(W)])
    for r in range(W):
        rk, ids, srcs, stt, sl, a = owner_side(batches, r)
        np.testing.assert_array_equal(res[r]["recv_keys"], rk)
        np.testing.assert_array_equal(res[r]["recv_idx"], ids)
        np.testing.assert_array_equal(res[r]["recv_src"], srcs)
        np.testing.assert_array_equal(res[r]["status"], stt)
        np.testing.assert_array_equal(res[r]["silo"], sl)
        np.testing.assert_array_equal(res[r]["act"], a)
        wp, wo = o.bucket_stable(a, n_act[r])
        np.testing.assert_array_equal(res[r]["perm"], wp)
        np.testing.assert_array_equal(res[r]["offsets"], wo)
        stt, sl, a, _, _ = o.route_batch_np(batches[r], spec, full, my_silo=r)
        np.testing.assert_array_equal(res[r]["ret_status"], stt)
        np.testing.assert_array_equal(res[r]["ret_silo"], sl)
        np.testing.assert_array_equal(res[r]["ret_act"], a)

    # the bench's timed mode: device batches, GD_MULTI_KEYS_READY | GD_MULTI_NO_KEYS, each result
    # read after the next batch was enqueued
    streams = [torch.cuda.Stream() for _ in range(W)]
    for r in range(W):
        es[r].set_stream(streams[r].cuda_stream)
    rounds = [[o.grain_keys(TC, zipf_ranks_np(G, sizes[r] // 2 + 1000 * i, 77 + 10 * r + i)) for i in range(3)]
              for r in range(W)]

    def read(rp, r):
        m = rp.n_recv
        v = lambda ptr, shape, t: _view(ptr, shape, t, "cuda").cpu().numpy()  # noqa: E731
        assert not rp.recv_keys                    # no key rebuild in this mode
        return {"recv_idx": v(rp.recv_idx, (m,), "<i4").view(np.uint32),
                "recv_src": v(rp.recv_src, (m,), "<i4").view(np.uint32),
                "status": v(rp.status, (m,), "|u1"), "silo": v(rp.silo, (m,), "<i4").view(np.uint32),
                "act": v(rp.act, (m,), "<i4").view(np.uint32), "perm": v(rp.perm, (m,), "<i4").view(np.uint32),
                "offsets": v(rp.offsets, (n_act[r] + 2,), "<i4").view(np.uint32)}

    def pipelined(r):
        dk = [torch.from_numpy(b.view(np.int64).copy()).cuda() for b in rounds[r]]
        torch.cuda.synchronize()
        got, prev = [], None
        for i in range(4):
            cur = None
            if i < 3:
                with torch.cuda.stream(streams[r]):
                    cur = es[r].route_multi_device(dk[i].data_ptr(), len(rounds[r][i]), n_act[r], keys_ready=True,
                                                   no_keys=True)
            if prev is not None:
                es[r].synchronize()
                got.append(read(prev, r))
            prev = cur
        return got

    res = _run_ranks([lambda r=r: pipelined(r) for r in range(W)])
    for i in range(3):
        for r in range(W):
            _, ids, srcs, stt, sl, a = owner_side([rounds[s][i] for s in range(W)], r)
            g_ = res[r][i]
            np.testing.assert_array_equal(g_["recv_idx"], ids, err_msg=f"batch {i} rank {r}")
            np.testing.assert_array_equal(g_["recv_src"], srcs)
            np.testing.assert_array_equal(g_["status"], stt)
            np.testing.assert_array_equal(g_["silo"], sl)
            np.testing.assert_array_equal(g_["act"], a)
            wp, wo = o.bucket_stable(a, n_act[r])
            np.testing.assert_array_equal(g_["perm"], wp)
            np.testing.assert_array_equal(g_["offsets"], wo)
    for e in es:
        e.comm_destroy()
        e.close()


# ----------------------------------------------------------------------------- histogram variants
@pytest.mark.parametrize("n,n_act", [(4097, 17), (12345, 256), (70001, 1 << 20), (5_000_003, 1 << 20),
                                     (5_000_003, 3_000_000)])
def test_bucket_hist_variants_unaligned(gd, monkeypatch, n, n_act):
    """The LSD path's radix histogram with 1 tile per workgroup (below 1,024 tiles) and 4 (5M
    messages), and the two-level forms' MSD histograms, on ragged sizes, from an activation array
    that starts 4 bytes past a 16-B boundary (the unaligned branch) and from an aligned one."""
    import torch
    rng = np.random.default_rng(n + 4)
    acts = rng.integers(0, n_act + n_act // 8 + 1, size=n).astype(np.uint32)
    acts[rng.random(n) < 0.01] = o.M32
    wp, wo = o.bucket_stable(acts, n_act)
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    e.set_stream(stream.cuda_stream)
    for shift in (1, 0):
        with torch.cuda.stream(stream):
            buf = torch.zeros(n + 4, dtype=torch.int32, device=dev)
            buf[shift:shift + n] = torch.from_numpy(acts.view(np.int32)).to(dev)
            perm = torch.empty(n, dtype=torch.int32, device=dev)
            off = torch.empty(n_act + 2, dtype=torch.int32, device=dev)
            e.bucket_device(buf.data_ptr() + 4 * shift, n, n_act, perm.data_ptr(), off.data_ptr())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(perm.cpu().numpy().view(np.uint32), wp, err_msg=f"shift {shift}")
        np.testing.assert_array_equal(off.cpu().numpy().view(np.uint32), wo)
    e.close()


# ----------------------------------------------------------------------------- packed radix records
@pytest.mark.parametrize("bucket", [0, 2])
@pytest.mark.parametrize("n,n_act,skew", [(70001, 1 << 20, False), (5_000_003, 1 << 20, True),
                                          (1 << 24, 1 << 20, False), (3_000_001, (1 << 16) + 5, False),
                                          (200_000, (1 << 23) + 3, True), (33_554_431, 1 << 20, False),
                                          (300_001, (1 << 24) - 5, False), (6_000_001, (1 << 24) - 5, True)])
def test_bucket_packed_records(gd, monkeypatch, bucket, n, n_act, skew):
    """The LSD passes (GD_OPT_BUCKET 0) pack records to 6 B between the passes where they fit: index
    and first digit in a u32, the higher key bits in a u16 that the later histograms read alone.  The
    shapes cover the u16 histogram with 1 and 4 tiles per workgroup, ragged tails, a u16 holding all
    16 bits (2^23 + 3 activations, 8-bit digits), an index and first digit filling all 32 bits
    (2^25 - 1 messages, 7-bit digits), unrouted messages and a hot key.  The same shapes through the
    two-level forms where they apply (GD_OPT_BUCKET 2: batches of 2^20 messages and up), against the
    oracle.  The 8-bit shapes end in 2^16-activation digit ranges that the one-launch range scan
    covers in 4 sub-ranges (most of them empty at 2^24 - 5)."""
    import torch
    monkeypatch.setitem(gd.DEFAULT_OPTIONS, "bucket", bucket)
    rng = np.random.default_rng(n ^ n_act)
    acts = rng.integers(0, n_act + n_act // 8 + 1, size=n).astype(np.uint32)
    if skew:
        acts[rng.random(n) < 0.3] = np.uint32(n_act // 3)
    acts[rng.random(n) < 0.01] = o.M32
    wp, wo = o.bucket_stable(acts, n_act)
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    dev = torch.device("cuda:0")
    stream = torch.cuda.Stream(dev)
    e.set_stream(stream.cuda_stream)
    with torch.cuda.stream(stream):
        a = torch.from_numpy(acts.view(np.int32)).to(dev)
        perm = torch.empty(n, dtype=torch.int32, device=dev)
        off = torch.empty(n_act + 2, dtype=torch.int32, device=dev)
        e.bucket_device(a.data_ptr(), n, n_act, perm.data_ptr(), off.data_ptr())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(perm.cpu().numpy().view(np.uint32), wp)
    np.testing.assert_array_equal(off.cpu().numpy().view(np.uint32), wo)
    e.close()


# ----------------------------------------------------------------------------- measured choices (GD_TUNE_*)
def test_tune_pin_get_reset(gd):
    """gd_tune_set pins a kind's variant from the first launch (the kernels that run show it), -1
    returns it to measuring, gd_tune_get reports the choice, gd_tune_reset forgets the measured ones;
    results never change."""
    acts = np.random.default_rng(3).integers(0, 1 << 20, size=1 << 21).astype(np.uint32)
    wp, wo = o.bucket_stable(acts, 1 << 20)
    q = (1 << 21) // ((1 << 20 >> 10) + 1)
    sub = 0
    while sub < 31 and (q >> sub) > 1:
        sub += 1
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    e.set_kernel_timing(True)
    for pin, want, absent in ((1, "k_msd_local", "k_starts_rangescan"), (0, "k_starts_rangescan", "k_msd_local")):
        e.tune_set("bucket", pin)
        assert e.tune_get("bucket", 1 << 21, sub) == pin
        e.kernel_times_reset()
        p, off = e.bucket(acts, 1 << 20)
        names = {k for k, (launches, _) in e.kernel_times().items() if launches}
        assert want in names and absent not in names, (pin, names)
        np.testing.assert_array_equal(p, wp)
        np.testing.assert_array_equal(off, wo)
    e.tune_set("bucket", -1)
    assert e.tune_get("bucket", 1 << 21, sub) == -1           # measuring
    for _ in range(6):                                         # 2 x 2 timed launches, then the pick
        p, off = e.bucket(acts, 1 << 20)
        np.testing.assert_array_equal(p, wp)
    assert e.tune_get("bucket", 1 << 21, sub) in (0, 1)
    e.tune_reset()
    assert e.tune_get("bucket", 1 << 21, sub) == -1
    with pytest.raises(gd.GrainDispatchError):
        e.tune_set("bucket", 2)                                # the bucketing has two variants
    e.close()


def test_tune_agree_w8(gd):
    """gd_tune_agree at W = 8 (in-process transport): after each rank measured its own probe and
    bucketing variants on live exchange batches, every rank keeps the same pick for every measured
    entry -- the variant with the least summed time -- and results stay bit-exact afterwards.  The
    communicator reports its 8 ranks (gd_comm_info)."""
    W, G = 8, 1 << 20
    # the bench's balanced silo set (every silo owns 1/8 of the ring): every rank receives a batch of
    # one size class, so the ranks measure the same tune entries
    gens = [138558, 165678, 215136, 61804, 17808, 48728, 207265, 76820]
    silos = [o.Silo(f"10.0.0.{i + 1}", 11111, gens[i]) for i in range(8)]
    spec = o.ring_spec(silos, "D")
    reg = o.grain_keys(TC, np.arange(G))
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    act = np.zeros(G, np.uint32)
    for r in range(W):
        act[own % W == r] = np.arange(int((own % W == r).sum()))
    n_act = [int((own % W == r).sum()) for r in range(W)]
    es = []
    for r in range(W):
        # the plain owner probe (its index / directory variants are what is measured)
        e = gd.GrainDispatch(device=0, table_capacity=1 << 19, my_silo=r, options={"region_probe": 0})
        e.ring_set_silos("D", _tuples(silos))
        mine = own % W == r
        e.register(reg[mine], act[mine], own[mine])
        es.append(e)
    gd.GrainDispatch.comm_init_local(es)
    for r in range(W):
        info = es[r].comm_info()
        assert info == {"n_ranks": W, "rank": r, "transport": "in-process"}, info
    rng = np.random.default_rng(88)
    n = 3 << 20
    batches = [o.grain_keys(TC, rng.integers(0, G, size=n)) for _ in range(W)]
    for _ in range(7):
        res = _run_ranks([lambda r=r: es[r].route_multi(batches[r], n_act[r], no_keys=True) for r in range(W)])
    m = [len(res[r]["act"]) for r in range(W)]
    assert len({int(x).bit_length() for x in m}) == 1            # one size class on every rank
    _run_ranks([lambda r=r: es[r].tune_agree() for r in range(W)])
    q = m[0] // ((n_act[0] >> 10) + 1)
    sub = 0
    while sub < 31 and (q >> sub) > 1:
        sub += 1
    for kind in ("probe_n1", "bucket"):
        picks = [es[r].tune_get(kind, m[r], sub if kind == "bucket" else 0) for r in range(W)]
        assert len(set(picks)) == 1 and picks[0] >= 0, (kind, picks)
    res = _run_ranks([lambda r=r: es[r].route_multi(batches[r], n_act[r]) for r in range(W)])
    full = o.DirectoryArrays(reg, act, own)
    for r in range(W):
        wp, wo = o.bucket_stable(res[r]["act"], n_act[r])
        np.testing.assert_array_equal(res[r]["perm"], wp)
        np.testing.assert_array_equal(res[r]["offsets"], wo)
        st, _, a, _, _ = o.route_batch_np(res[r]["recv_keys"], spec, full, my_silo=r)
        np.testing.assert_array_equal(res[r]["act"], a)
    for e in es:
        e.comm_destroy()
        e.close()


def test_tune_agree_rank_without_8b_index(gd):
    """gd_tune_agree when one rank's 8-B probe index cannot hold one of its entries (N1 >= 2^32 on rank
    0) and that rank never measured the agreed entry: ranks 1..3 time their 24-B-key probe variants (the
    8-B index among them) on a size class rank 0 never routes, the agreement hands rank 0 a pick for that
    entry, and rank 0's launches of that size run it with results equal to the oracle's.  (Rounds 4-5:
    such an entry kept rank 0 from building the 8-B index at all, and the pick had to be re-measured
    there; round 6 builds it on every rank and probes the keys it does not hold in the directory, so
    any agreed variant is one rank 0 has.)"""
    W, G = 4, 1 << 16
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    reg = o.grain_keys(TC, np.arange(G))
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    wide = o.grain_keys(TC, np.array([0], dtype=np.int64))
    wide[0, 1] = np.uint64(1 << 33)                          # N1 >= 2^32: no 8-B index on rank 0
    wide_own = o.ring_owner_np(spec, o.jenkins_u64x3_np(wide[:, 2], wide[:, 0], wide[:, 1])).astype(np.uint32)
    es = []
    for r in range(W):
        e = gd.GrainDispatch(device=0, table_capacity=1 << 17, my_silo=r)
        e.ring_set_silos("D", _tuples(silos))
        e.register(reg, np.arange(G, dtype=np.uint32), own)
        if r == 0:
            e.register(wide, np.array([G], np.uint32), wide_own)
        es.append(e)
    gd.GrainDispatch.comm_init_local(es)
    rng = np.random.default_rng(5)
    keys = o.grain_keys(TC, rng.integers(0, G, size=1 << 20))
    for r in range(1, W):                                    # 8 launches: every variant timed twice
        for _ in range(10):
            es[r].route(keys)
    _run_ranks([lambda r=r: es[r].tune_agree() for r in range(W)])
    picks = [es[r].tune_get("probe_keys", len(keys)) for r in range(1, W)]
    assert len(set(picks)) == 1 and picks[0] >= 0, picks
    full = o.DirectoryArrays(np.concatenate([reg, wide]), np.arange(G + 1, dtype=np.uint32),
                             np.concatenate([own, wide_own]))
    want = o.route_batch_np(keys, spec, full)
    for _ in range(10):                                      # measuring again over rank 0's own variants
        st, silo, act = es[0].route(keys)
        np.testing.assert_array_equal(st, want[0])
        np.testing.assert_array_equal(silo, want[1])
        np.testing.assert_array_equal(act, want[2])
    assert es[0].tune_get("probe_keys", len(keys)) in (-1, 0, 1, 2, 3)
    assert es[0].index_stats()["out8"] >= 1                  # the N1 >= 2^32 entry: not in the 8-B index
    for e in es:
        e.comm_destroy()
        e.close()


def test_stable_rank_fallback_without_lane_order(gd):
    """A handle on a device without the LDS lane order (GD_CFG_NO_LANE_ORDER stands in for a failed
    gd_create check) is created, ranks by ballots (GD_OPT_STABLE_RANK reads 0) and refuses 1."""
    e = gd.GrainDispatch(device=0, table_capacity=1 << 12, no_lane_order=True)
    assert e.get_option("stable_rank") == 0
    with pytest.raises(Exception):
        e.set_option("stable_rank", 1)
    assert e.get_option("stable_rank") == 0
    e.close()


def test_options_roundtrip_and_range(gd, monkeypatch):
    """gd_option_set / gd_option_get: every option reads back what was set, the defaults are the
    documented ones, values out of range and unknown options are refused with an error
    (the handle keeps its value)."""
    monkeypatch.setattr(gd, "DEFAULT_OPTIONS", {})           # the library's own defaults, not this module's
    e = gd.GrainDispatch(device=0, table_capacity=1 << 12)   # creation ran the lane-order self-check
    defaults = {"probe": 1, "bucket": 1, "l2_small": 1024, "stable_rank": 0 if gd.FORCE_NO_LANE_ORDER else 1,
                "wire_headers": 2,
                "region_probe": 0, "idx16": 1, "host_chunk": 2097152, "mb_zerocopy": 1, "mb_split": 8,
                "mb_trace": 0, "l2_staged": 24576, "l2_mid": 8192, "b2_persist": 2, "b2_order": 0, "mb_poll": 1,
                "fan_bound": 0}
    assert set(defaults) == set(gd.OPTIONS)
    for k, v in defaults.items():
        assert e.get_option(k) == v, k
    for k, v in {"probe": 4, "bucket": 2, "l2_small": 300, "stable_rank": 0, "wire_headers": 0,
                 "region_probe": 1, "idx16": 0, "l2_staged": 9000, "l2_mid": 2000, "b2_persist": 0,
                 "b2_order": 1, "mb_poll": 0, "fan_bound": 1}.items():
        e.set_option(k, v)
        assert e.get_option(k) == v, k
    for k, bad in {"probe": 5, "bucket": -1, "l2_small": 24577, "l2_mid": 8193, "l2_staged": 1 << 20,
                   "b2_persist": 9, "b2_order": 2, "mb_poll": 2, "fan_bound": 2}.items():
        before = e.get_option(k)
        with pytest.raises(Exception):
            e.set_option(k, bad)
        assert e.get_option(k) == before, k
    with pytest.raises(Exception):
        e.set_option(99, 1)
    e.close()


def test_comm_info_world1_rccl(gd):
    """gd_comm_info reports the communicator as RCCL sees it: none before gd_comm_init, one rank over
    RCCL after, none again after gd_comm_destroy."""
    e = gd.GrainDispatch(device=0, table_capacity=1 << 12)
    assert e.comm_info()["transport"] == "none"
    e.comm_init(gd.GrainDispatch.comm_unique_id(), 1, 0)
    assert e.comm_info() == {"n_ranks": 1, "rank": 0, "transport": "rccl"}
    e.comm_destroy()
    assert e.comm_info()["transport"] == "none"
    e.close()
