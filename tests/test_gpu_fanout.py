"""GPU parity for the follower fan-out (BASELINE cfg 4) through the C ABI,
against oracle/fanout.py.  Every integer output is compared bit for bit."""
import numpy as np
import pytest

import fanout as fo
from orleans_amd.workloads import power_law_graph
import oracle as o

pytestmark = pytest.mark.gpu

TC = o.grain_type_code(fo.CHIRPER_ACCOUNT_CLASS)


@pytest.fixture(scope="module")
def gd():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from orleans_amd import graindispatch as g
    return g


def _setup(gd, n_nodes, mode="D", registered=None, cap=None, probe=None):
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, mode)
    reg_nodes = np.arange(n_nodes) if registered is None else np.asarray(registered)
    reg = o.grain_keys(TC, reg_nodes)
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    e = gd.GrainDispatch(device=0, table_capacity=cap or max(1024, 2 * len(reg_nodes)),
                         options=None if probe is None else {"probe": probe})
    e.ring_set_silos(mode, [(s.ip, s.port, s.gen) for s in silos])
    e.register(reg, reg_nodes.astype(np.uint32), owner)
    d = o.DirectoryArrays(reg, reg_nodes.astype(np.uint32), owner)
    return e, spec, d


def _want_hop(ro, dst, frontier, spec, d, n_act):
    t, s = fo.expand(ro, dst, frontier)
    st, silo, act, _, _ = o.route_batch_np(o.grain_keys(TC, t.astype(np.int64)), spec, d)
    perm, off = o.bucket_stable(act, n_act)
    return dict(target=t, sender=s, status=st, silo=silo, act=act, perm=perm, offsets=off)


@pytest.mark.parametrize("mode,probe", [("D", None), ("R", None), ("V", None), ("D", 0), ("D", 2), ("V", 4)])
def test_fanout_hop_vs_oracle(gd, mode, probe):
    """probe: the route's probe forced (0 directory, 2 the 16-B index, 4 the 8-B index), None measured."""
    n = 6000
    ro, dst = power_law_graph(n, 8.0, seed=11, max_deg=3000)
    rng = np.random.default_rng(12)
    registered = np.sort(rng.choice(n, size=int(n * 0.95), replace=False))     # 5% MISS
    e, spec, d = _setup(gd, n, mode, registered, probe=probe)
    frontier = np.concatenate([rng.integers(0, n, 700), [3, 3, 3], [n, n + 5, 0xFFFFFFF0]]).astype(np.uint32)
    got = e.fanout_route_bucket(ro, dst, frontier, TC, n)
    want = _want_hop(ro, dst, frontier, spec, d, n)
    assert got["target"].size == want["target"].size > 0
    for k in want:
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    assert (got["status"] == o.ST_MISS).any()
    # without bucketing
    got2 = e.fanout_route_bucket(ro, dst, frontier, TC, None)
    np.testing.assert_array_equal(got2["act"], want["act"])
    e.close()


def test_fan_bound_launch_leaves_results(gd):
    """GD_OPT_FAN_BOUND (bench.py's live bound of k_fan_route): each 8-B-index fan-out route is preceded by
    k_fan_bound on the same inputs into scratch; the hop's outputs stay the oracle's, and both kernels are
    timed once a hop."""
    n = 6000
    ro, dst = power_law_graph(n, 8.0, seed=13, max_deg=3000)
    rng = np.random.default_rng(14)
    e, spec, d = _setup(gd, n, "D", probe=4)
    e.set_option("fan_bound", 1)
    e.set_kernel_timing(1)
    e.kernel_times_reset()
    for _ in range(2):
        frontier = rng.integers(0, n, 900).astype(np.uint32)
        got = e.fanout_route_bucket(ro, dst, frontier, TC, n)
        want = _want_hop(ro, dst, frontier, spec, d, n)
        for k in want:
            np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    t = e.kernel_times()
    e.set_kernel_timing(False)
    assert t["k_fan_bound"][0] == t["k_fan_route"][0] == 2
    e.set_option("fan_bound", 0)
    e.close()


def _device(gd, e):
    import torch
    from orleans_amd.fanout import DeviceFanoutEngine
    return DeviceFanoutEngine(e, torch.device("cuda", 0), TC)


def test_fanout_expand_load_balance_edges(gd):
    """A celebrity row far longer than a block's tile, and a run of zero-follower publishers
    longer than the block's LDS staging (the global-search fallback)."""
    import torch
    from orleans_amd.fanout import upload_graph
    n = 40000
    rows = [[] for _ in range(n)]
    rng = np.random.default_rng(5)
    rows[7] = list(rng.choice(n, size=30000, replace=False))                  # celebrity
    for u in range(20000, 20100):
        rows[u] = list(rng.choice(n, size=3, replace=False))
    rows[39999] = [1, 2]
    ro, dst = fo.csr_from_rows(rows)
    e, spec, d = _setup(gd, n)
    eng = _device(gd, e)
    g = upload_graph(ro, dst, eng.device)
    fronts = [
        np.array([7], np.uint32),
        np.arange(20000, 20100, dtype=np.uint32),
        np.concatenate([[7], np.arange(100, 12000), [20050], np.arange(12000, 19990), [39999]]).astype(np.uint32),
        np.arange(100, 9000, dtype=np.uint32),                                   # all zero-degree
        np.zeros(0, np.uint32),
        np.array([20001, 7, 20001, 7, 39999] * 3, np.uint32),
    ]
    with eng.context():
        for fr in fronts:
            t, s = eng.expand(g, torch.from_numpy(fr.view(np.int32)).to(eng.device))
            wt, ws = fo.expand(ro, dst, fr)
            np.testing.assert_array_equal(t.cpu().numpy().view(np.uint32), wt)
            np.testing.assert_array_equal(s.cpu().numpy().view(np.uint32), ws)
            got = e.fanout_route_bucket(ro, dst, fr, TC, n)
            want = _want_hop(ro, dst, fr, spec, d, n)
            for k in want:
                np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    e.close()


@pytest.mark.parametrize("mode", ["D", "V"])
def test_cascade_device_vs_oracle(gd, mode):
    import torch
    from orleans_amd.fanout import FanoutCascade, upload_graph
    n = 30000
    ro, dst = power_law_graph(n, 6.0, seed=21, max_deg=5000)
    rng = np.random.default_rng(22)
    registered = np.sort(rng.choice(n, size=int(n * 0.98), replace=False))
    e, spec, d = _setup(gd, n, mode, registered)
    eng = _device(gd, e)
    g = upload_graph(ro, dst, eng.device)
    seeds = rng.integers(0, n, 100).astype(np.uint32)
    hops = FanoutCascade(eng, g, n).run(torch.from_numpy(seeds.view(np.int32)).to(eng.device), 4)
    want = fo.cascade(ro, dst, seeds, 4, spec, d, n, TC)
    assert sum(w["target"].size for w in want) > 10000
    for h, (gh, wh) in enumerate(zip(hops, want)):
        u = lambda t: t.cpu().numpy().view(np.uint32)  # noqa: E731
        np.testing.assert_array_equal(u(gh.frontier), wh["frontier"], err_msg=f"hop {h} frontier")
        for k in ("target", "sender", "silo", "act", "perm", "offsets"):
            np.testing.assert_array_equal(u(getattr(gh, k)), wh[k], err_msg=f"hop {h} {k}")
        np.testing.assert_array_equal(gh.status.cpu().numpy(), wh["status"], err_msg=f"hop {h} status")
    e.close()


@pytest.mark.parametrize("probe", [None, 0, 4])
def test_route_nodes_pack_and_frontier_vs_oracle(gd, probe):
    """probe: the node route's probe forced (0 directory, 4 the 8-B index), None measured."""
    import torch
    n = 50000
    e, spec, d = _setup(gd, n, "D", np.arange(0, n, 2), probe=probe)   # odd nodes unregistered
    eng = _device(gd, e)
    rng = np.random.default_rng(9)
    nodes = rng.integers(0, n + 100, 100000).astype(np.uint32)
    payload = np.arange(nodes.size, dtype=np.uint32) * 7
    tn = torch.from_numpy(nodes.view(np.int32)).to(eng.device)
    tp = torch.from_numpy(payload.view(np.int32)).to(eng.device)
    with eng.context():
        st, silo, act, perm, off = eng.route_nodes_bucket(tn, n)
        w = o.route_batch_np(o.grain_keys(TC, nodes.astype(np.int64)), spec, d)
        np.testing.assert_array_equal(st.cpu().numpy(), w[0])
        np.testing.assert_array_equal(silo.cpu().numpy().view(np.uint32), w[1])
        np.testing.assert_array_equal(act.cpu().numpy().view(np.uint32), w[2])
        wp, wo = o.bucket_stable(w[2], n)
        np.testing.assert_array_equal(perm.cpu().numpy().view(np.uint32), wp)
        np.testing.assert_array_equal(off.cpu().numpy().view(np.uint32), wo)
        for shards in (1, 3, 8):
            sn, sp, counts = eng.pack_nodes_by_shard(tn, tp, shards)
            dest = (w[3] % shards).astype(np.uint32)
            p2, o2 = o.bucket_stable(dest, shards)
            np.testing.assert_array_equal(sn.cpu().numpy().view(np.uint32), nodes[p2])
            np.testing.assert_array_equal(sp.cpu().numpy().view(np.uint32), payload[p2])
            np.testing.assert_array_equal(counts.cpu().numpy(), np.diff(o2[:shards + 1]))
        # frontier: visited preset on a third of the activations
        visited = np.zeros(n, dtype=bool)
        visited[::3] = True
        tv = torch.from_numpy(visited.astype(np.uint8)).to(eng.device)
        fr = eng.frontier_next(off, n, tv)
        vis2 = visited.copy()
        wf = fo.next_frontier(wo, n, vis2)
        np.testing.assert_array_equal(fr.cpu().numpy().view(np.uint32), wf)
        np.testing.assert_array_equal(tv.cpu().numpy().astype(bool), vis2)
    e.close()


def test_cascade_large_properties(gd):
    """2M-node power-law graph, 3 hops: size-independent properties (every message is a
    follower edge of its publisher, counts add up, per-activation order is stable, frontiers
    are new and distinct) plus an oracle check of a sample of hop 1."""
    import torch
    from orleans_amd.fanout import FanoutCascade, upload_graph
    n = 1 << 21
    ro, dst = power_law_graph(n, 10.0, seed=31, max_deg=1 << 16)
    e, spec, d = _setup(gd, n, "D", cap=1 << 23)
    eng = _device(gd, e)
    g = upload_graph(ro, dst, eng.device)
    rng = np.random.default_rng(32)
    seeds = np.unique(rng.integers(0, n, 2000)).astype(np.uint32)
    hops = FanoutCascade(eng, g, n).run(torch.from_numpy(seeds.view(np.int32)).to(eng.device), 3)
    seen = np.zeros(n, dtype=bool)
    seen[seeds] = True
    ro64 = ro.astype(np.int64)
    total = 0
    for h, hr in enumerate(hops):
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
        assert (st == o.ST_OK).all() and np.array_equal(act, t)          # every node registered, act = node
        np.testing.assert_array_equal(np.repeat(fr, deg), s)             # publisher order, degree each
        # message k of publisher i is its k-th follower
        starts = np.repeat(ro64[fr] - np.concatenate([[0], np.cumsum(deg)[:-1]]), deg)
        np.testing.assert_array_equal(dst[starts + np.arange(t.size)], t)
        # bucketing: sorted by activation, stable
        assert (np.diff(act[perm].astype(np.int64)) >= 0).all()
        same = np.diff(act[perm].astype(np.int64)) == 0
        assert (np.diff(perm.astype(np.int64))[same] > 0).all()
        assert off[-1] == t.size and off[n] == t.size
        if h:
            assert not seen[fr].any() and np.unique(fr).size == fr.size
            seen[fr] = True
    assert total > 1_000_000
    # oracle on a sample of hop 1's publishers
    fr1 = hops[1].frontier.cpu().numpy().view(np.uint32)[:300]
    want = _want_hop(ro, dst, fr1, spec, d, n)
    got = e.fanout_route_bucket(ro, dst, fr1, TC, n)
    for k in want:
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)
    e.close()
