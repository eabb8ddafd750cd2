"""The receive-path oracle (oracle/receive.py): the vectorised restatement equals the
literal per-message loop of IncomingMessageAgent.ReceiveMessage, including the overload rule, and
hand-built cases follow the reference branches."""
import numpy as np
import pytest

import oracle as o
import receive as rv

TC = o.grain_type_code(o.PING_GRAIN_CLASS)


def _act_ids(rng, m):
    k = np.zeros((m, 3), np.uint64)
    k[:, 0] = rng.integers(0, 1 << 63, size=m, dtype=np.int64).astype(np.uint64)
    k[:, 1] = rng.integers(0, 1 << 63, size=m, dtype=np.int64).astype(np.uint64)
    return k


def _world(seed, n_act=300, n_st=20, n=5000):
    rng = np.random.default_rng(seed)
    aid = _act_ids(rng, n_act)
    st_keys = np.zeros((n_st, 3), np.uint64)
    st_keys[:, 1] = np.arange(n_st, dtype=np.uint64) + 7
    st_keys[:, 2] = np.uint64(o.type_code_data(o.CAT_SYSTEM_TARGET, 12))
    keys = np.concatenate([aid, st_keys])
    ctxs = np.arange(n_act + n_st, dtype=np.uint32)
    flags = np.concatenate([np.where(rng.random(n_act) < 0.9, rv.AD_VALID, 0) |
                            np.where(rng.random(n_act) < 0.2, rv.AD_STATELESS_WORKER, 0),
                            np.full(n_st, rv.AD_SYSTEM_TARGET | rv.AD_VALID)]).astype(np.uint32)
    # messages: app grains to known / unknown activations, system targets known / unknown,
    # and cross-kind lookups (an app grain naming a system target's activation id and back)
    which = rng.integers(0, n_act + n_st + 40, size=n)
    ta = np.zeros((n, 3), np.uint64)
    tg = o.grain_keys(TC, rng.integers(0, 1000, size=n))
    known = which < n_act + n_st
    ta[known] = keys[which[known]]
    ta[~known] = _act_ids(rng, int((~known).sum()))
    sys_msg = (which >= n_act) & (which < n_act + n_st) | (rng.random(n) < 0.02)
    cross = rng.random(n) < 0.03
    sys_msg = np.where(cross, ~sys_msg, sys_msg)
    tg[sys_msg, 2] = np.uint64(o.type_code_data(o.CAT_SYSTEM_TARGET, 12))
    direction = rng.choice([0, 1, 2, 0xFF, 7], size=n, p=[0.5, 0.2, 0.2, 0.08, 0.02]).astype(np.uint8)
    ad = rv.ActivationDirectory()
    for k, c, f in zip(keys, ctxs, flags):
        assert ad.add(tuple(int(x) for x in k), int(c), int(f))
    return rng, keys, ctxs, flags, tg, ta, direction, ad, n_act + n_st


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("limits", [None, (3, 2), (1, 0), (0, 5)])
def test_receive_np_equals_loop(seed, limits):
    rng, keys, ctxs, flags, tg, ta, direction, ad, n_ctx = _world(seed)
    rc = None if limits is None else rng.integers(0, 5, size=n_ctx)
    hl, hls = (0, 0) if limits is None else limits
    want = rv.receive_batch(tg, ta, direction, ad, n_ctx, rc, hl, hls)
    got = rv.receive_batch_np(tg, ta, direction, keys, ctxs, flags, n_ctx, rc, hl, hls)
    for w, g in zip(want, got):
        np.testing.assert_array_equal(g, w)
    assert set(np.unique(want[0])) >= {rv.RECV_ACTIVATION, rv.RECV_SYSTEM_TARGET, rv.RECV_NULL_CONTEXT,
                                       rv.RECV_REJECT_UNKNOWN, rv.RECV_DROPPED}
    if limits is not None and limits[0] > 0:
        assert (want[0] == rv.RECV_REJECT_OVERLOADED).any()


def test_receive_reference_branches():
    """One message per branch of IncomingMessageAgent.ReceiveMessage (:92-170)."""
    ad = rv.ActivationDirectory()
    a_valid, a_inval, st = (1, 2, 0), (3, 4, 0), (0, 9, o.type_code_data(o.CAT_SYSTEM_TARGET, 5))
    ad.add(a_valid, 0, rv.AD_VALID)
    ad.add(a_inval, 1, 0)
    ad.add(st, 2, rv.AD_SYSTEM_TARGET | rv.AD_VALID)
    assert not ad.add(a_valid, 5, 0)                    # TryAdd: first wins
    app = o.grain_keys(TC, [1])[0]
    stg = np.array(st, np.uint64)
    rows = [(app, a_valid, 0, rv.RECV_ACTIVATION, 0), (app, a_valid, 1, rv.RECV_ACTIVATION, 0),
            (app, a_inval, 0, rv.RECV_NULL_CONTEXT, 3), (app, (5, 5, 0), 0, rv.RECV_NULL_CONTEXT, 3),
            (app, st, 0, rv.RECV_NULL_CONTEXT, 3),                            # FindTarget ignores systemTargets
            (stg, st, 0, rv.RECV_SYSTEM_TARGET, 2), (stg, st, 1, rv.RECV_SYSTEM_TARGET, 2),
            (stg, st, 2, rv.RECV_DROPPED, rv.M32), (stg, st, 0xFF, rv.RECV_SYSTEM_TARGET, 2),
            (stg, a_valid, 0, rv.RECV_REJECT_UNKNOWN, rv.M32)]
    tg = np.array([r[0] for r in rows], np.uint64)
    ta = np.array([r[1] for r in rows], np.uint64)
    d = np.array([r[2] for r in rows], np.uint8)
    status, ctx, perm, off = rv.receive_batch(tg, ta, d, ad, 3)
    assert status.tolist() == [r[3] for r in rows]
    assert ctx.tolist() == [r[4] for r in rows]
    assert perm.tolist() == [0, 1, 5, 6, 8, 2, 3, 4, 7, 9]
    assert off.tolist() == [0, 2, 2, 5, 8, 10]
    # overload: hard limit 2, activation 0 starts at count 1: request (count 1 ok -> 2), response
    # (always, -> 3), request (3 > 2: rejected), response (-> 4), one-way (rejected)
    d = np.array([0, 1, 0, 1, 2], np.uint8)
    s, c, _, _ = rv.receive_batch(np.repeat(app[None], 5, 0), np.repeat(np.array(a_valid, np.uint64)[None], 5, 0),
                                  d, ad, 3, request_count=[1, 0, 0], hard_limit=2)
    assert s.tolist() == [0, 0, 4, 0, 4]
    assert not ad.remove((9, 9, 9)) and ad.remove(a_inval)
