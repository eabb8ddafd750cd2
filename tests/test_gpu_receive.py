"""GPU parity for the receive path: the ActivationDirectory table and
IncomingMessageAgent.ReceiveMessage (IncomingMessageAgent.cs:92-170) with per-context bucketing,
through the C ABI, against oracle/receive.py -- from key arrays, from device arrays at 4M messages,
and straight from frames; plus gd_route_frames bucketing addressed frames by their TargetActivation."""
import numpy as np
import pytest

import headers as H
import oracle as o
import receive as rv

pytestmark = pytest.mark.gpu

TC = o.grain_type_code(o.PING_GRAIN_CLASS)


@pytest.fixture(scope="module")
def gd():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from orleans_amd import graindispatch as g
    return g


def _act_ids(rng, m):
    k = np.zeros((m, 3), np.uint64)
    k[:, 0] = rng.integers(1, 1 << 62, size=m, dtype=np.int64).astype(np.uint64)
    k[:, 1] = rng.integers(0, 1 << 62, size=m, dtype=np.int64).astype(np.uint64)
    return k


def _world(seed, n_act, n_st, n):
    """Activations + system targets in one context space, and a message batch that hits every
    branch: known / unknown / invalid activations, known / unknown system targets, cross-kind ids,
    all directions incl. absent (0xFF) and undefined values."""
    rng = np.random.default_rng(seed)
    aid = _act_ids(rng, n_act)
    st_keys = np.zeros((n_st, 3), np.uint64)
    st_keys[:, 1] = np.arange(n_st, dtype=np.uint64) + 7
    st_keys[:, 2] = np.uint64(o.type_code_data(o.CAT_SYSTEM_TARGET, 12))
    keys = np.concatenate([aid, st_keys])
    ctxs = rng.permutation(n_act + n_st).astype(np.uint32)
    flags = np.concatenate([np.where(rng.random(n_act) < 0.9, rv.AD_VALID, 0) |
                            np.where(rng.random(n_act) < 0.2, rv.AD_STATELESS_WORKER, 0),
                            np.full(n_st, rv.AD_SYSTEM_TARGET | rv.AD_VALID)]).astype(np.uint8)
    which = rng.integers(0, n_act + n_st + max(1, (n_act + n_st) // 8), size=n)
    ta = np.zeros((n, 3), np.uint64)
    tg = o.grain_keys(TC, rng.integers(0, 1000, size=n))
    known = which < n_act + n_st
    ta[known] = keys[which[known]]
    ta[~known] = _act_ids(rng, int((~known).sum()))
    sys_msg = ((which >= n_act) & known) | (rng.random(n) < 0.02)
    cross = rng.random(n) < 0.03
    sys_msg = np.where(cross, ~sys_msg, sys_msg)
    tg[sys_msg, 2] = np.uint64(o.type_code_data(o.CAT_SYSTEM_TARGET, 12))
    direction = rng.choice([0, 1, 2, 0xFF, 7], size=n, p=[0.5, 0.2, 0.2, 0.08, 0.02]).astype(np.uint8)
    return rng, keys, ctxs, flags, tg, ta, direction


@pytest.mark.parametrize("limits", [None, (3, 2), (0, 4)])
def test_receive_vs_oracle(gd, limits):
    rng, keys, ctxs, flags, tg, ta, direction = _world(5, 3000, 40, 60000)
    n_ctx = len(keys)
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    added = e.actdir_add(keys, ctxs, flags)
    assert added.all() and e.actdir_count() == n_ctx
    rc = None if limits is None else rng.integers(0, 6, size=n_ctx).astype(np.uint32)
    hl, hls = (0, 0) if limits is None else limits
    ctx, st, perm, off = e.receive(tg, ta, direction, n_ctx, rc, hl, hls)
    ad = rv.ActivationDirectory()
    for k, c, f in zip(keys, ctxs, flags):
        ad.add(tuple(int(x) for x in k), int(c), int(f))
    w = rv.receive_batch(tg, ta, direction, ad, n_ctx, rc, hl, hls)
    np.testing.assert_array_equal(st, w[0])
    np.testing.assert_array_equal(ctx, w[1])
    np.testing.assert_array_equal(perm, w[2])
    np.testing.assert_array_equal(off, w[3])
    assert {int(x) for x in np.unique(st)} >= {0, 1, 2, 3, 5} | ({4} if hl else set())
    # no direction array: every message a Request
    ctx2, st2 = e.receive(tg, ta, None, n_ctx, bucket=False)
    w2 = rv.receive_batch(tg, ta, np.zeros(len(tg), np.uint8), ad, n_ctx)
    np.testing.assert_array_equal(st2, w2[0])
    np.testing.assert_array_equal(ctx2, w2[1])
    # limits without buckets: CheckOverloaded still applies (it used to be skipped)
    ctx3, st3 = e.receive(tg, ta, direction, n_ctx, rc, hl, hls, bucket=False)
    np.testing.assert_array_equal(st3, w[0])
    np.testing.assert_array_equal(ctx3, w[1])
    assert int(st3.max()) <= 6                     # no transient stateless-worker mark leaks out
    e.close()


def test_receive_context_out_of_range(gd):
    """An ActivationDirectory entry whose context index is not below the call's n_ctx is a caller
    error (GD_EINVAL), never an out-of-bounds read of request_count / offsets."""
    rng, keys, ctxs, flags, tg, ta, direction = _world(7, 500, 8, 4000)
    n_ctx = len(keys)
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    e.actdir_add(keys, ctxs, flags)
    rc = np.zeros(n_ctx - 100, np.uint32)
    with pytest.raises(gd.GrainDispatchError):
        e.receive(tg, ta, direction, n_ctx - 100, rc, 3, 2)
    # the handle stays usable, and a correct n_ctx routes as before
    ctx, st, perm, off = e.receive(tg, ta, direction, n_ctx)
    ad = rv.ActivationDirectory()
    for k, c, f in zip(keys, ctxs, flags):
        ad.add(tuple(int(x) for x in k), int(c), int(f))
    w = rv.receive_batch(tg, ta, direction, ad, n_ctx)
    np.testing.assert_array_equal(st, w[0])
    np.testing.assert_array_equal(perm, w[2])
    e.close()


def test_actdir_ops_vs_oracle(gd):
    """TryAdd (first wins, in-batch duplicates), TryRemove, state changes (last wins), lookups,
    growth past the initial table."""
    rng = np.random.default_rng(9)
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    ad = rv.ActivationDirectory()
    ids = _act_ids(rng, 6000)
    for step in range(12):
        k = int(rng.integers(1, 3000))
        sel = rng.integers(0, len(ids), size=k)
        op = step % 3
        if op == 0:
            ctx = rng.integers(0, 1 << 20, size=k).astype(np.uint32)
            fl = rng.integers(0, 8, size=k).astype(np.uint8)
            got = e.actdir_add(ids[sel], ctx, fl)
            want = [ad.add(tuple(int(x) for x in ids[s]), int(c), int(f)) for s, c, f in zip(sel, ctx, fl)]
            np.testing.assert_array_equal(got, want)
        elif op == 1:
            got = e.actdir_remove(ids[sel])
            want = [ad.remove(tuple(int(x) for x in ids[s])) for s in sel]
            np.testing.assert_array_equal(got, want)
        else:
            fl = rng.integers(0, 8, size=k).astype(np.uint8)
            got = e.actdir_set_flags(ids[sel], fl)
            want = [ad.set_flags(tuple(int(x) for x in ids[s]), int(f)) for s, f in zip(sel, fl)]
            np.testing.assert_array_equal(got, want)
        c, f, found = e.actdir_lookup(ids)
        for i in range(len(ids)):
            w = ad.entries.get(tuple(int(x) for x in ids[i]))
            assert bool(found[i]) == (w is not None)
            if w is not None:
                assert (c[i], f[i]) == w
        assert e.actdir_count() == len(ad.entries)
    e.actdir_clear()
    assert e.actdir_count() == 0
    e.close()


def test_receive_device_4m(gd):
    """4,194,304 messages over 1M activations from device arrays, with overload limits, against the
    vectorised oracle."""
    import torch
    rng, keys, ctxs, flags, tg, ta, direction = _world(17, 1 << 20, 64, 1 << 22)
    n_ctx = len(keys)
    n = len(tg)
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    e.actdir_add(keys, ctxs, flags)
    rc = rng.integers(0, 4, size=n_ctx).astype(np.uint32)
    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    e.set_stream(s.cuda_stream)
    with torch.cuda.stream(s):
        d_tg = torch.from_numpy(tg.view(np.int64)).to(dev)
        d_ta = torch.from_numpy(ta.view(np.int64)).to(dev)
        d_dir = torch.from_numpy(direction).to(dev)
        d_rc = torch.from_numpy(rc.view(np.int32)).to(dev)
        ctx = torch.empty(n, dtype=torch.int32, device=dev)
        st = torch.empty(n, dtype=torch.uint8, device=dev)
        perm = torch.empty(n, dtype=torch.int32, device=dev)
        off = torch.empty(n_ctx + 3, dtype=torch.int32, device=dev)
        e.receive_device(d_tg.data_ptr(), d_ta.data_ptr(), d_dir.data_ptr(), n, n_ctx, ctx.data_ptr(), st.data_ptr(),
                         perm.data_ptr(), off.data_ptr(), d_rc.data_ptr(), 2, 1)
    torch.cuda.synchronize()
    w = rv.receive_batch_np(tg, ta, direction, keys, ctxs, flags, n_ctx, rc, 2, 1)
    np.testing.assert_array_equal(st.cpu().numpy(), w[0])
    np.testing.assert_array_equal(ctx.cpu().numpy().view(np.uint32), w[1])
    np.testing.assert_array_equal(perm.cpu().numpy().view(np.uint32), w[2])
    np.testing.assert_array_equal(off.cpu().numpy().view(np.uint32), w[3])
    e.close()


def _frames_for(tg, ta, direction, rng, p_incomplete=0.05, p_fallback=0.02):
    """Addressed request/response frames (TargetGrain + TargetActivation + TargetSilo), some without
    the activation (not addressed), some with an object-serialized field first (fallback)."""
    parts, offs, pos = [], [], 0
    silo = (b"\x00" * 12 + bytes([10, 0, 0, 2]), 11111, 3)
    for i in range(len(tg)):
        h = {"category": 2, "correlation_id": i + 1, "target_grain": (tuple(int(x) for x in tg[i]), None)}
        if direction[i] != 0xFF:
            h["direction"] = int(direction[i])
        if rng.random() >= p_incomplete:
            h["target_activation"] = (tuple(int(x) for x in ta[i]), None)
            h["target_silo"] = silo
        if rng.random() < 0.3:
            h["sending_grain"] = ((0, i, int(tg[i][2])), None)
        if rng.random() < p_fallback:
            h["request_context"] = b"\x01\x00\x00\x00" + bytes(12)
        fr = H.encode_frame(h, bytes(int(rng.integers(0, 40))))
        parts.append(fr)
        offs.append(pos)
        pos += len(fr)
    return b"".join(parts), np.array(offs, np.uint64)


def test_receive_frames_vs_oracle(gd):
    rng, keys, ctxs, flags, tg, ta, direction = _world(23, 2000, 30, 15000)
    direction[direction == 7] = 2                 # the frame's Direction byte as written
    n_ctx = len(keys)
    buf, off = _frames_for(tg, ta, direction, rng)
    e = gd.GrainDispatch(device=0, table_capacity=1024)
    e.actdir_add(keys, ctxs, flags)
    dec, ctx, st, perm, offs = e.receive_frames(buf, off, n_ctx, fields=["target_activation", "direction"])
    f = H.decode_frames(buf, off)
    np.testing.assert_array_equal(dec["target_activation"], f["target_activation"])
    np.testing.assert_array_equal(dec["direction"], f["direction"])
    ok = ((f["flags"] & H.F_HAS_TARGET) != 0) & ((f["flags"] & H.F_COMPLETE) != 0) & \
         ((f["flags"] & (H.F_FALLBACK | H.F_MALFORMED)) == 0)
    ad = rv.ActivationDirectory()
    for k, c, fl in zip(keys, ctxs, flags):
        ad.add(tuple(int(x) for x in k), int(c), int(fl))
    w = rv.receive_batch(f["target_grain"], f["target_activation"], f["direction"], ad, n_ctx)
    wst, wctx = w[0].copy(), w[1].copy()
    wst[~ok] = 6                                   # GD_RECV_UNDECODED: back to the C# deserializer
    wctx[~ok] = rv.M32
    np.testing.assert_array_equal(st, wst)
    np.testing.assert_array_equal(ctx, wctx)
    key = np.where(wctx != rv.M32, wctx.astype(np.int64), n_ctx + 1)
    np.testing.assert_array_equal(perm, np.argsort(key, kind="stable"))
    np.testing.assert_array_equal(offs[1:], np.cumsum(np.bincount(key, minlength=n_ctx + 2)))
    assert (~ok).sum() > 0 and (st == rv.RECV_ACTIVATION).sum() > 0
    e.close()


def test_route_frames_addressed_use_activation_directory(gd):
    """gd_route_frames with an ActivationDirectory: addressed frames (complete address, not looked
    up) land in their activation's bucket when FindTarget finds it Valid; the rest as before."""
    G = 3000
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    reg = o.grain_keys(TC, np.arange(G))
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    e = gd.GrainDispatch(device=0, table_capacity=1 << 13, my_silo=3, seed_silo=5)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    e.register(reg, np.arange(G), owner)
    rng = np.random.default_rng(2)
    aid = _act_ids(rng, G)                         # activation g of grain g has ActivationId aid[g]
    valid = rng.random(G) < 0.8
    e.actdir_add(aid, np.arange(G, dtype=np.uint32), np.where(valid, rv.AD_VALID, 0).astype(np.uint8))
    n = 8000
    gi = rng.integers(0, G, size=n)
    tg = reg[gi]
    ta = aid[gi]
    ta[rng.random(n) < 0.05] = _act_ids(rng, 1)[0]   # a stale activation id
    buf, off = _frames_for(tg, ta, np.zeros(n, np.uint8), rng, p_incomplete=0.5)
    dec, st, silo, act, perm, offs = e.route_frames(buf, off, n_act=G)
    f, wst, wsilo, wact = H.route_frames_np(buf, off, spec, o.DirectoryArrays(reg, np.arange(G), owner))
    wst2, wsilo2, wact2 = o.route_batch_np(f["target_grain"], spec, o.DirectoryArrays(reg, np.arange(G), owner),
                                           my_silo=3, seed_silo=5)[:3]
    routed = wst < H.ROUTE_ADDRESSED
    wst[routed], wsilo[routed], wact[routed] = wst2[routed], wsilo2[routed], wact2[routed]
    ad = {tuple(int(x) for x in aid[g]): g for g in range(G) if valid[g]}
    for i in np.nonzero(wst == H.ROUTE_ADDRESSED)[0]:
        wact[i] = ad.get(tuple(int(x) for x in f["target_activation"][i]), rv.M32)
    np.testing.assert_array_equal(st, wst)
    np.testing.assert_array_equal(silo, wsilo)
    np.testing.assert_array_equal(act, wact)
    wp, wo = o.bucket_stable(wact, G)
    np.testing.assert_array_equal(perm, wp)
    np.testing.assert_array_equal(offs, wo)
    assert ((st == H.ROUTE_ADDRESSED) & (act != rv.M32)).sum() > 0
    e.close()
