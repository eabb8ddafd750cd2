"""GPU parity for the sharded fan-out cascade behind the C ABI (gd_fanout_multi*, BASELINE cfg 4
across GPUs: SURVEY 8 f2 over 8 e) against oracle/fanout.py, and cfg 4 at its BASELINE size.

* W = 8 (and 3) ranks on one GPU through the in-process transport (gd_comm_init_local): every
  hop's frontier, owner-side arrival order (sender rank, sender emission order), routes, buckets.
* W = 1 over RCCL: the sharded cascade equals the one-GPU fused cascade bit for bit.
* cfg 4 at full size (10M grains, ~100M follower edges, 65,536 seeds, 3 hops) on one GPU:
  size-independent properties of every hop plus an oracle sample of each hop.
Reference: Samples/Chirper/ChirperGrains/ChirperAccount.cs:106-147 (publish loop :131-134)."""
import numpy as np
import pytest

import fanout as fo
import oracle as o
from orleans_amd.workloads import power_law_graph

pytestmark = pytest.mark.gpu

TC = o.grain_type_code(fo.CHIRPER_ACCOUNT_CLASS)


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


def _owners_of(spec, nodes):
    reg = o.grain_keys(TC, np.asarray(nodes, dtype=np.int64))
    return o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)


def _owners(spec, n):
    return _owners_of(spec, np.arange(n))


@pytest.mark.parametrize("W,mode", [(8, "D"), (3, "V")])
def test_fanout_multi_local_world_vs_oracle(gd, W, mode):
    n, hops = 20000, 4
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, mode)
    ro, dst = power_law_graph(n, 6.0, seed=41 + W, max_deg=4000)
    own = _owners(spec, n)
    registered = np.arange(n)[np.arange(n) % 23 != 4]              # some followers have no activation
    es = []
    for r in range(W):
        e = gd.GrainDispatch(device=0, table_capacity=1 << 14, my_silo=r)
        e.ring_set_silos(mode, [(s.ip, s.port, s.gen) for s in silos])
        mine = registered[own[registered] % W == r]
        e.register(o.grain_keys(TC, mine), mine.astype(np.uint32), own[mine])
        es.append(e)
    gd.GrainDispatch.comm_init_local(es)
    seeds = np.random.default_rng(W).integers(0, n, 40).astype(np.uint32)
    seeds = np.concatenate([seeds, seeds[:3], [n + 7]]).astype(np.uint32)   # duplicates, a node past the graph
    res = _run_ranks([lambda r=r: es[r].fanout_multi(ro, dst, seeds, TC, n, hops) for r in range(W)])
    full = o.DirectoryArrays(o.grain_keys(TC, registered), registered.astype(np.uint32), own[registered])
    want = fo.cascade(ro, dst, seeds, hops, spec, full, n, TC)
    own_rank = own % W
    assert sum(w["target"].size for w in want) > 20000
    for h in range(hops):
        fronts = [res[r][h]["frontier"] for r in range(W)]
        if h == 0:
            seed_rank = _owners_of(spec, seeds) % W
            for r in range(W):       # each rank publishes the seeds it owns, in seed order (duplicates too)
                assert fronts[r].tolist() == seeds[seed_rank == r].tolist(), (h, r)
        else:
            assert sorted(np.concatenate(fronts).tolist()) == want[h]["frontier"].tolist(), h
            for r in range(W):
                assert (own_rank[fronts[r]] == r).all()
                assert (np.diff(fronts[r].astype(np.int64)) > 0).all()
        for r in range(W):
            tt, ss, src = [], [], []
            for q in range(W):
                t, s = fo.expand(ro, dst, fronts[q])
                keep = own_rank[t] == r
                tt.append(t[keep]), ss.append(s[keep]), src.append(np.full(int(keep.sum()), q, np.uint32))
            t, s = np.concatenate(tt), np.concatenate(ss)
            got = res[r][h]
            np.testing.assert_array_equal(got["target"], t, err_msg=f"hop {h} rank {r} target")
            np.testing.assert_array_equal(got["sender"], s, err_msg=f"hop {h} rank {r} sender")
            np.testing.assert_array_equal(got["src"], np.concatenate(src), err_msg=f"hop {h} rank {r} src")
            assert got["n_sent"] == fo.expand(ro, dst, fronts[r])[0].size
            st, silo, act, _, _ = o.route_batch_np(o.grain_keys(TC, t.astype(np.int64)), spec, full, my_silo=r)
            np.testing.assert_array_equal(got["status"], st, err_msg=f"hop {h} rank {r} status")
            np.testing.assert_array_equal(got["silo"], silo)
            np.testing.assert_array_equal(got["act"], act)
            wp, wo = o.bucket_stable(act, n)
            np.testing.assert_array_equal(got["perm"], wp, err_msg=f"hop {h} rank {r} perm")
            np.testing.assert_array_equal(got["offsets"], wo, err_msg=f"hop {h} rank {r} offsets")
        assert sum(res[r][h]["target"].size for r in range(W)) == want[h]["target"].size
    for e in es:
        e.comm_destroy()
        e.close()


def test_fanout_multi_partitioned_graph_w8(gd):
    """The cascade over a partitioned follower graph (gd_fanout_multi_part_device): each of W = 8
    in-process ranks holds only the rows of the grains it owns (~1/8 of the edges), its directory
    maps each owned node to its local row.  Every hop equals the replicated-graph cascade's (itself
    checked against the oracle above): frontier, target, sender, sending rank, status, silo, and
    each activation's message list (perm slice) mapped row -> node."""
    import torch
    from orleans_amd.fanout import partition_graph_np
    W, n, hops = 8, 20000, 4
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    ro, dst = power_law_graph(n, 6.0, seed=77, max_deg=4000)
    own = _owners(spec, n)
    registered = np.arange(n)[np.arange(n) % 23 != 4]
    rep, part, parts = [], [], []
    dev = torch.device("cuda", 0)
    for r in range(W):
        mine = registered[own[registered] % W == r]
        a = gd.GrainDispatch(device=0, table_capacity=1 << 14, my_silo=r)
        a.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
        a.register(o.grain_keys(TC, mine), mine.astype(np.uint32), own[mine])
        rep.append(a)
        b = gd.GrainDispatch(device=0, table_capacity=1 << 14, my_silo=r)
        b.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
        b.register(o.grain_keys(TC, mine), np.arange(mine.size, dtype=np.uint32), own[mine])
        part.append(b)
        ro_l, dst_l, node_of = partition_graph_np(ro, dst, mine)
        parts.append(tuple(torch.from_numpy(x.view(np.int32)).to(dev) if x.size else
                           torch.zeros(1, dtype=torch.int32, device=dev) for x in (ro_l, dst_l, node_of)) +
                     (mine.size, dst_l.size))
    # each rank: its owned grains' rows only (the owner share of the literal generation-1 silo set peaks
    # at ~36 %); every stored edge once over the ranks
    assert max(p[4] for p in parts) < 0.45 * dst.size and sum(p[4] for p in parts) <= dst.size
    gd.GrainDispatch.comm_init_local(rep)
    gd.GrainDispatch.comm_init_local(part)
    seeds = np.random.default_rng(8).choice(registered, 60).astype(np.uint32)
    seeds = np.concatenate([seeds, seeds[:3]]).astype(np.uint32)                  # duplicates
    t_seeds = torch.from_numpy(seeds.view(np.int32)).to(dev)
    torch.cuda.synchronize()
    want = _run_ranks([lambda r=r: rep[r].fanout_multi(ro, dst, seeds, TC, n, hops) for r in range(W)])

    def run_part(r):
        ro_d, dst_d, no_d, rows, _ = parts[r]
        hr = part[r].fanout_multi_part_device(ro_d.data_ptr(), dst_d.data_ptr(), rows, no_d.data_ptr(),
                                              t_seeds.data_ptr(), seeds.size, TC, hops)
        out = [part[r].fanout_multi_fetch(h, hr[h], rows) for h in range(hops)]
        part[r].synchronize()
        return out
    got = _run_ranks([lambda r=r: run_part(r) for r in range(W)])
    assert sum(want[r][h]["target"].size for r in range(W) for h in range(hops)) > 20000
    for r in range(W):
        node_of = parts[r][2].cpu().numpy().view(np.uint32)[:parts[r][3]]
        for h in range(hops):
            g, w = got[r][h], want[r][h]
            for k in ("frontier", "target", "sender", "src", "status", "silo"):
                np.testing.assert_array_equal(g[k], w[k], err_msg=f"hop {h} rank {r} {k}")
            assert g["n_sent"] == w["n_sent"]
            ok = g["status"] == 0
            np.testing.assert_array_equal(node_of[g["act"][ok]], w["act"][ok], err_msg=f"hop {h} rank {r} act")
            for i, u in enumerate(node_of):                       # each activation's messages, in order
                np.testing.assert_array_equal(g["perm"][g["offsets"][i]:g["offsets"][i + 1]],
                                              w["perm"][w["offsets"][u]:w["offsets"][u + 1]],
                                              err_msg=f"hop {h} rank {r} row {i}")
            rows = parts[r][3]
            np.testing.assert_array_equal(g["perm"][g["offsets"][rows]:], w["perm"][w["offsets"][n]:],
                                          err_msg=f"hop {h} rank {r} unrouted")
    for e in rep + part:
        e.comm_destroy()
        e.close()


def test_fanout_multi_partitioned_bad_seed_fails_on_every_rank(gd):
    """A seed without a live activation on its owner (a partitioned graph's rows are activations)
    fails gd_fanout_multi_part_device on EVERY rank, together, after hop 0's counts round -- no rank
    is left waiting in a later exchange round (W = 4, in-process transport).  The handles stay usable:
    the next cascade with valid seeds runs on all ranks."""
    import torch
    from orleans_amd.fanout import partition_graph_np
    W, n, hops = 4, 4000, 3
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    ro, dst = power_law_graph(n, 5.0, seed=91, max_deg=500)
    own = _owners(spec, n)
    registered = np.arange(n)[np.arange(n) % 17 != 3]
    dev = torch.device("cuda", 0)
    es, parts = [], []
    for r in range(W):
        mine = registered[own[registered] % W == r]
        e = gd.GrainDispatch(device=0, table_capacity=1 << 12, my_silo=r)
        e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
        e.register(o.grain_keys(TC, mine), np.arange(mine.size, dtype=np.uint32), own[mine])
        es.append(e)
        ro_l, dst_l, node_of = partition_graph_np(ro, dst, mine)
        parts.append(tuple(torch.from_numpy(x.view(np.int32)).to(dev) if x.size else
                           torch.zeros(1, dtype=torch.int32, device=dev) for x in (ro_l, dst_l, node_of)) +
                     (mine.size,))
    gd.GrainDispatch.comm_init_local(es)
    good = np.random.default_rng(3).choice(registered, 20).astype(np.uint32)
    bad = np.concatenate([good, [3]]).astype(np.uint32)          # node 3 has no activation
    assert own[3] % W in range(W)

    def run(r, seeds):
        t = torch.from_numpy(seeds.view(np.int32)).to(dev)
        torch.cuda.synchronize()
        ro_d, dst_d, no_d, rows = parts[r]
        try:
            es[r].fanout_multi_part_device(ro_d.data_ptr(), dst_d.data_ptr(), rows, no_d.data_ptr(), t.data_ptr(),
                                           seeds.size, TC, hops)
            return None
        except Exception as ex:   # noqa: BLE001 -- the error is the result here
            return str(ex)
    errs = _run_ranks([lambda r=r: run(r, bad) for r in range(W)])
    for r in range(W):
        assert errs[r] is not None and "no live activation" in errs[r], (r, errs[r])
        assert f"rank {int(own[3] % W)}" in errs[r], (r, errs[r])
    errs = _run_ranks([lambda r=r: run(r, good) for r in range(W)])
    assert errs == [None] * W, errs
    for e in es:
        e.comm_destroy()
        e.close()


def test_fanout_multi_world1_rccl_equals_fused_cascade(gd):
    """W = 1 over RCCL (a send/recv to self): the sharded cascade gives exactly the one-GPU fused
    cascade's hops (same emission order, same frontiers)."""
    import torch
    from orleans_amd.fanout import DeviceFanoutEngine, FanoutCascade, upload_graph
    n, hops = 200000, 3
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    ro, dst = power_law_graph(n, 8.0, seed=5, max_deg=20000)
    own = _owners(spec, n)
    e = gd.GrainDispatch(device=0, table_capacity=1 << 19, my_silo=0)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    e.register(o.grain_keys(TC, np.arange(n)), np.arange(n, dtype=np.uint32), own)
    e.comm_init(gd.GrainDispatch.comm_unique_id(), 1, 0)
    dev = torch.device("cuda", 0)
    eng = DeviceFanoutEngine(e, dev, TC)
    g = upload_graph(ro, dst, dev)
    seeds = np.unique(np.random.default_rng(6).integers(0, n, 500)).astype(np.uint32)
    t_seeds = torch.from_numpy(seeds.view(np.int32)).to(dev)
    with eng.context():
        hr = e.fanout_multi_device(g.row_off.data_ptr(), g.dst.data_ptr(), n, t_seeds.data_ptr(), seeds.size, TC, n,
                                   hops)
        got = [e.fanout_multi_fetch(h, hr[h], n) for h in range(hops)]
        ref = FanoutCascade(eng, g, n).run(t_seeds, hops)
    eng.synchronize()
    u = lambda t: t.cpu().numpy().view(np.uint32)  # noqa: E731
    assert sum(x["target"].size for x in got) > 100000
    for h in range(hops):
        np.testing.assert_array_equal(got[h]["frontier"], u(ref[h].frontier), err_msg=f"hop {h}")
        for k in ("target", "sender", "silo", "act", "perm", "offsets"):
            np.testing.assert_array_equal(got[h][k], u(getattr(ref[h], k)), err_msg=f"hop {h} {k}")
        np.testing.assert_array_equal(got[h]["status"], ref[h].status.cpu().numpy())
        assert (got[h]["src"] == 0).all() and got[h]["n_sent"] == got[h]["target"].size
    e.comm_destroy()
    e.close()


def test_library_cascade_equals_host_driven_cascade(gd):
    """gd_fanout_cascade_device (the one-GPU cascade inside the library, one read-back a hop) gives
    exactly the host-driven cascade's hops (FanoutCascade: gd_fanout_route_bucket_device +
    gd_frontier_next_device per hop): frontiers, targets, senders, routes, buckets."""
    import torch
    from orleans_amd.fanout import DeviceFanoutEngine, FanoutCascade, LibraryCascade, upload_graph
    n, hops = 200000, 4
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    ro, dst = power_law_graph(n, 8.0, seed=15, max_deg=20000)
    own = _owners(spec, n)
    e = gd.GrainDispatch(device=0, table_capacity=1 << 19, my_silo=0)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    reg = np.arange(n)[np.arange(n) % 17 != 3]                   # some followers have no activation
    e.register(o.grain_keys(TC, reg), reg.astype(np.uint32), own[reg])
    dev = torch.device("cuda", 0)
    eng = DeviceFanoutEngine(e, dev, TC)
    g = upload_graph(ro, dst, dev)
    lc = LibraryCascade(eng, g, n)
    u = lambda t: t.cpu().numpy().view(np.uint32)  # noqa: E731
    rng = np.random.default_rng(16)
    # the first cascade sizes the hop buffers; the repeat routes each hop before its size is read back
    # (k_fan_route reading the size on the device); a larger seed set outgrows them, a smaller one fits
    for rep, n_seeds in enumerate((700, 700, 2500, 90)):
        seeds = np.unique(rng.choice(reg, n_seeds)).astype(np.uint32) if rep != 1 else seeds
        t_seeds = torch.from_numpy(seeds.view(np.int32)).to(dev)
        got = lc.fetch(lc.run(t_seeds, hops))
        ref = FanoutCascade(eng, g, n).run(t_seeds, hops)
        eng.synchronize()
        if rep < 2:
            assert sum(x["target"].size for x in got) > 100000
        for h in range(hops):
            np.testing.assert_array_equal(got[h]["frontier"], u(ref[h].frontier), err_msg=f"rep {rep} hop {h}")
            for k in ("target", "sender", "silo", "act", "perm", "offsets"):
                np.testing.assert_array_equal(got[h][k], u(getattr(ref[h], k)), err_msg=f"rep {rep} hop {h} {k}")
            np.testing.assert_array_equal(got[h]["status"], ref[h].status.cpu().numpy())
            assert (got[h]["src"] == 0).all()
    e.close()


def test_library_cascade_large_hops_repeat(gd):
    """The in-library cascade at hop sizes past the small-tile bound (2,048-output tiles), run twice on
    one handle (the repeat routes before the read-back), against the host-driven cascade."""
    import torch
    from orleans_amd.fanout import DeviceFanoutEngine, FanoutCascade, LibraryCascade, upload_graph
    n, hops = 2_000_000, 3
    silos = o.bench_silos(8)
    ro, dst = power_law_graph(n, 10.0, seed=25, max_deg=1 << 16)
    e = gd.GrainDispatch(device=0, table_capacity=1 << 23, my_silo=0)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    keys = o.grain_keys(TC, np.arange(n))
    e.register(keys, np.arange(n, dtype=np.uint32), e.ring_owner(keys))
    del keys
    dev = torch.device("cuda", 0)
    eng = DeviceFanoutEngine(e, dev, TC)
    g = upload_graph(ro, dst, dev)
    seeds = np.random.default_rng(26).choice(n, size=1 << 14, replace=False).astype(np.uint32)
    t_seeds = torch.from_numpy(seeds.view(np.int32)).to(dev)
    lc = LibraryCascade(eng, g, n)
    ref = FanoutCascade(eng, g, n).run(t_seeds, hops)
    eng.synchronize()
    assert max(int(r.target.shape[0]) for r in ref) > 4_000_000
    for rep in range(2):
        got = lc.fetch(lc.run(t_seeds, hops))
        for h in range(hops):
            assert got[h]["target"].size == int(ref[h].target.shape[0])
            for k in ("frontier", "target", "sender", "silo", "act", "perm", "offsets"):
                want = u32_np(getattr(ref[h], k))
                assert np.array_equal(got[h][k], want), f"rep {rep} hop {h} {k}"
            assert np.array_equal(got[h]["status"], ref[h].status.cpu().numpy())
    e.close()


def u32_np(t):
    return t.cpu().numpy().view(np.uint32)


def test_cfg4_full_size_properties(gd):
    """BASELINE cfg 4 at its size on one GPU: 10M grains, ~100M follower edges (power law, mean 10,
    cap 65,536; the bench's graph), 65,536 seeds, 3 hops.  Size-independent properties of every hop
    (each message is a follower edge of its publisher in enumeration order, counts add up, buckets
    sorted and stable, frontiers new and distinct) plus the oracle on a sample of each hop's
    publishers."""
    import torch
    from orleans_amd.fanout import DeviceFanoutEngine, FanoutCascade, upload_graph
    n, hops = 10_000_000, 3
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    ro, dst = power_law_graph(n, 10.0, seed=0x5EED0004, max_deg=1 << 16)
    assert ro[-1] > 90_000_000
    e = gd.GrainDispatch(device=0, table_capacity=1 << 25, my_silo=0)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    keys = o.grain_keys(TC, np.arange(n))
    owner = e.ring_owner(keys)
    e.register(keys, np.arange(n, dtype=np.uint32), owner)
    del keys
    dev = torch.device("cuda", 0)
    eng = DeviceFanoutEngine(e, dev, TC)
    g = upload_graph(ro, dst, dev)
    seeds = np.random.default_rng(0x5EED0004).choice(n, size=1 << 16, replace=False).astype(np.uint32)
    hops_r = FanoutCascade(eng, g, n).run(torch.from_numpy(seeds.view(np.int32)).to(dev), hops)
    eng.synchronize()
    seen = np.zeros(n, dtype=bool)
    seen[seeds] = True
    ro64 = ro.astype(np.int64)
    total = 0
    samples = []
    for h, hr in enumerate(hops_r):
        fr = hr.frontier.cpu().numpy().view(np.uint32)
        t = hr.target.cpu().numpy().view(np.uint32)
        s = hr.sender.cpu().numpy().view(np.uint32)
        act = hr.act.cpu().numpy().view(np.uint32)
        st = hr.status.cpu().numpy()
        perm = hr.perm.cpu().numpy().view(np.uint32)
        off = hr.offsets.cpu().numpy().view(np.uint32)
        deg = ro64[fr.astype(np.int64) + 1] - ro64[fr]
        assert t.size == int(deg.sum())
        total += t.size
        assert (st == o.ST_OK).all() and np.array_equal(act, t)          # every grain registered, act = node
        np.testing.assert_array_equal(np.repeat(fr, deg), s)             # publisher order, degree each
        starts = np.repeat(ro64[fr] - np.concatenate([[0], np.cumsum(deg)[:-1]]), deg)
        np.testing.assert_array_equal(dst[starts + np.arange(t.size)], t)
        sa = act[perm].astype(np.int64)
        assert (np.diff(sa) >= 0).all()
        assert (np.diff(perm.astype(np.int64))[np.diff(sa) == 0] > 0).all()
        cnt = np.bincount(act, minlength=n + 1)
        np.testing.assert_array_equal(np.diff(off[:n + 1].astype(np.int64)), cnt[:n])
        assert off[n] == t.size and off[n + 1] == t.size
        if h:
            assert not seen[fr].any() and np.unique(fr).size == fr.size and (np.diff(fr.astype(np.int64)) > 0).all()
            seen[fr] = True
        samples.append(fr[:: max(1, fr.size // 200)][:200])
        del t, s, act, st, perm, off
    assert total > 40_000_000
    # the oracle on a sample of each hop's publishers (the directory restricted to the grains they reach)
    for h, fs in enumerate(samples):
        t, s = fo.expand(ro, dst, fs)
        nodes = np.unique(t)
        d = o.DirectoryArrays(o.grain_keys(TC, nodes), nodes.astype(np.uint32), owner[nodes])
        want = dict(zip(("status", "silo", "act"), o.route_batch_np(o.grain_keys(TC, t.astype(np.int64)), spec, d)[:3]))
        got = e.fanout_route_bucket(ro, dst, fs, TC, None)
        np.testing.assert_array_equal(got["target"], t, err_msg=f"hop {h}")
        np.testing.assert_array_equal(got["sender"], s)
        for k in want:
            np.testing.assert_array_equal(got[k], want[k], err_msg=f"hop {h} {k}")
    e.close()
