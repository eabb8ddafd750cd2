"""GPU parity for the multi-rank directory handoff behind the C ABI (gd_dir_handoff_multi, SURVEY 8 f4
over 8 e) against oracle/dirstate.py, at W = 8 ranks on one GPU through the in-process transport.

* Silo removal (GrainDirectoryHandoffManager.ProcessSiloRemoveEvent, :125-158): the leaver's entries
  move to their new owners and are merged there (GrainDirectoryPartition.Merge :497-522,
  GrainInfo.Merge :139-179): absent -> inserted with the sender's VersionTag and SingleInstance flag,
  a competing single activation -> the lowest ActivationId stays and the loser is reported for
  Catalog.DeleteActivations, the same ActivationId -> unchanged, multi-activation -> the host's.
* Silo join (ProcessSiloAddEvent, :195-245): entries the newcomer now owns move to it and are
  registered there (RegisterMany(singleActivation: true): the first registration wins).
Afterwards every rank's partition equals the oracle's, VersionTags included."""
import numpy as np
import pytest

import dirstate as ds
import oracle as o

pytestmark = pytest.mark.gpu

TC = o.grain_type_code(o.PING_GRAIN_CLASS)
W = 8


@pytest.fixture(scope="module")
def gd():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from orleans_amd import graindispatch as g
    return g


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


def _ring(mode, silos, members):
    """Ring of the member silos, owners as original silo indices (AddServer over them)."""
    spec = o.ring_spec([silos[i] for i in members], mode)
    return o.RingSpec(spec.mode, spec.points, [members[x] for x in spec.owners])


def _owner(spec, keys):
    return o.ring_owner_np(spec, o.jenkins_u64x3_np(keys[:, 2], keys[:, 0], keys[:, 1])).astype(np.uint32)


def _set_ring(e, mode, spec):
    e.ring_set(mode, np.asarray(spec.points, np.int64) if mode != "V" else np.asarray(spec.points, np.uint32),
               np.asarray(spec.owners, np.uint32))


def _ids(rng, m):
    k = np.zeros((m, 3), np.uint64)
    k[:, 0] = rng.integers(1, 1 << 62, size=m, dtype=np.int64).astype(np.uint64)
    k[:, 1] = rng.integers(0, 1 << 62, size=m, dtype=np.int64).astype(np.uint64)
    return k


def _check_state(e, st, universe):
    act, silo, tag, found = e.lookup_tagged(universe)
    want = st.lookup_tagged(universe)
    np.testing.assert_array_equal(found, [w[3] for w in want])
    np.testing.assert_array_equal(act, [w[0] for w in want])
    np.testing.assert_array_equal(silo, [w[1] for w in want])
    np.testing.assert_array_equal(tag, [w[2] for w in want])
    assert e.stats()["table_live"] == len(st.entries)


@pytest.mark.parametrize("event,mode", [("remove", "D"), ("remove", "V"), ("add", "D"), ("add", "V")])
def test_handoff_multi_local_world(gd, event, mode):
    silos = o.bench_silos(8)
    G = 16000
    reg = o.grain_keys(TC, np.arange(G))
    rng = np.random.default_rng({("remove", "D"): 31, ("remove", "V"): 32, ("add", "D"): 33, ("add", "V"): 34}[(event, mode)])
    changed = 3 if event == "remove" else 7
    before = list(range(8)) if event == "remove" else [s for s in range(8) if s != changed]
    after = [s for s in range(8) if s != changed] if event == "remove" else list(range(8))
    spec0, spec1 = _ring(mode, silos, before), _ring(mode, silos, after)
    own0, own1 = _owner(spec0, reg), _owner(spec1, reg)
    es, sts, n_idx, gid = [], [], [], {}
    ids_all = _ids(rng, 3 * G)
    for r in range(W):
        e = gd.GrainDispatch(device=0, table_capacity=1 << 14, my_silo=r)
        _set_ring(e, mode, spec0)
        st = ds.DirectoryState()
        mine = np.nonzero(own0 % W == r)[0]
        acts = np.arange(len(mine), dtype=np.uint32)          # this rank's activation indices
        ids = ids_all[mine]
        e.activation_ids_set(acts, ids)
        st.set_ids(acts, ids)
        multi = mine[::97] if r == changed or event == "add" else mine[:0]
        single = np.setdiff1d(mine, multi)
        pos = {g: i for i, g in enumerate(mine)}
        sa = np.array([pos[g] for g in single], np.uint32)
        if len(single):
            e.register(reg[single], sa, own0[single])
            st.register(reg[single], sa, own0[single])
        if len(multi):                                     # AddActivation grains (GD_ACT_MULTI entries)
            e.upsert(reg[multi], np.full(len(multi), ds.ACT_MULTI, np.uint32), own0[multi])
            st.upsert(reg[multi], np.full(len(multi), ds.ACT_MULTI, np.uint32), own0[multi])
        for g in mine:
            gid[int(g)] = tuple(int(x) for x in ids_all[g])
        es.append(e)
        sts.append(st)
        n_idx.append(len(mine))
    # receivers already hold some moving grains: a competing activation (lower or higher ActivationId)
    # or the very same ActivationId under another index
    moving = np.nonzero((own1 % W) != (own0 % W))[0]
    assert len(moving) > 40
    for r in range(W):
        comp = moving[(own1[moving] % W == r)][::4]
        if not len(comp):
            continue
        cids = _ids(rng, len(comp))
        same = np.arange(len(comp)) % 5 == 0
        cids[same] = ids_all[comp[same]]
        lower = np.arange(len(comp)) % 5 == 1
        cids[lower, 0] = 0                                 # N0 = 0 < every original's N0: these sort lower
        cids[~lower & ~same, 2] = np.uint64(1)             # TypeCodeData 1 > 0: these sort higher
        cacts = np.arange(n_idx[r], n_idx[r] + len(comp), dtype=np.uint32)
        es[r].activation_ids_set(cacts, cids)
        sts[r].set_ids(cacts, cids)
        csilo = np.full(len(comp), r, np.uint32)
        es[r].register(reg[comp], cacts, csilo)
        sts[r].register(reg[comp], cacts, csilo)
        n_idx[r] += len(comp)
    gd.GrainDispatch.comm_init_local(es)
    for e in es:
        _set_ring(e, mode, spec1)
    ev = gd.GD_HANDOFF_REMOVE if event == "remove" else gd.GD_HANDOFF_ADD
    keep = [[s for s in after if s % W == r] for r in range(W)]
    res = _run_ranks([lambda r=r: es[r].handoff_multi(keep[r], 8, ev, n_idx[r]) for r in range(W)])
    # the oracle: senders lose what they no longer own, in their partition's (any) order
    new_owner = lambda k: int(own1[k[1]])  # noqa: E731  (grain g is [0, g, tcd])
    sent = {}
    for q in range(W):
        lost = [k for k in sts[q].entries if new_owner(k) not in keep[q]]
        sent[q] = {k: sts[q].entries.pop(k) for k in lost}
        assert res[q]["n_sent"] == len(lost)
    statuses = set()
    for r in range(W):
        got = res[r]
        m = len(got["keys"])
        src = got["src"]
        assert (np.diff(src.astype(np.int64)) >= 0).all()
        keys = [tuple(int(x) for x in k) for k in got["keys"]]
        for q in range(W):
            want_keys = {k for k in sent[q] if new_owner(k) % W == r}
            assert {k for k, s in zip(keys, src) if s == q} == want_keys, (r, q)
        if not m:
            continue
        acts = np.where([sent[q][k][0] == ds.ACT_MULTI for k, q in zip(keys, src)], ds.ACT_MULTI,
                        n_idx[r] + np.arange(m)).astype(np.uint32)
        np.testing.assert_array_equal(got["act"], acts)
        silos_in = np.array([sent[q][k][1] for k, q in zip(keys, src)], np.uint32)
        np.testing.assert_array_equal(got["silo"], silos_in)
        for j, (k, q) in enumerate(zip(keys, src)):
            if acts[j] != ds.ACT_MULTI:
                assert tuple(int(x) for x in got["ids"][j]) == sts[q].ids[sent[q][k][0]]
        single_acts = [(int(a), sts[q].ids[sent[q][k][0]]) for a, k, q in zip(acts, keys, src) if a != ds.ACT_MULTI]
        sts[r].set_ids([a for a, _ in single_acts], [i for _, i in single_acts])
        if event == "remove":
            tags = [sent[q][k][2] | (0 if sent[q][k][3] else 0x80000000) for k, q in zip(keys, src)]
            want = sts[r].merge(keys, acts, silos_in, tags)
        else:
            want = sts[r].register_handoff(keys, acts, silos_in)
        bad = [(j, int(got["status"][j]), tuple(int(x) for x in got["dropped"][j]), want[j]) for j in range(m)
               if (int(got["status"][j]), int(got["dropped"][j][0]), int(got["dropped"][j][1])) != tuple(want[j])]
        assert not bad, (r, bad[:8])           # (position, status, dropped) vs the oracle
        np.testing.assert_array_equal(got["status"], [w[0] for w in want], err_msg=f"rank {r}")
        np.testing.assert_array_equal(got["dropped"][:, 0], [w[1] for w in want], err_msg=f"rank {r}")
        np.testing.assert_array_equal(got["dropped"][:, 1], [w[2] for w in want], err_msg=f"rank {r}")
        statuses |= {int(x) for x in got["status"]}
    expect = {ds.MERGE_INSERTED, ds.MERGE_SAME, ds.MERGE_DROPPED, ds.MERGE_HOST}
    if event == "remove":
        expect |= {ds.MERGE_KEPT}
    if len(moving) > 500:                              # every branch taken (the D ring moves few grains on a join)
        assert statuses >= expect, statuses
    for r in range(W):
        _check_state(es[r], sts[r], reg)
    for e in es:
        e.comm_destroy()
        e.close()
