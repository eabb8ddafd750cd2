"""CPU checks of the fan-out oracle: State.Followers enumeration order under
AddFollower / RemoveFollower (ChirperAccount.cs:213-232 with .NET Dictionary slot reuse), the
publish expansion (ChirperAccount.cs:131-134) and the cascade frontier rule."""
import numpy as np

import fanout as f
from orleans_amd.workloads import power_law_graph
import oracle as o


def test_followers_dictionary_order():
    d = f.FollowersDict()
    for k in (10, 11, 12):
        d.add_follower(k)
    assert d.values() == [10, 11, 12]
    d.remove(11)
    d.add_follower(13)                 # takes the slot 11 freed
    assert d.values() == [10, 13, 12]
    d.add_follower(10)                 # re-follow: Remove + add lands in the same slot
    assert d.values() == [10, 13, 12]
    d.remove(10)
    d.remove(12)                       # free list: 12's slot (head), then 10's
    d.add_follower(14)
    d.add_follower(15)
    assert d.values() == [15, 13, 14]
    d.add_follower(16)                 # free list empty: append
    assert d.values() == [15, 13, 14, 16]
    assert not d.remove(99)


def test_build_follower_csr():
    ops = [(0, 5, 1), (0, 6, 1), (2, 0, 1), (0, 7, 1), (0, 6, -1), (0, 8, 1), (3, 3, -1)]
    ro, dst = f.build_follower_csr(4, ops)
    assert ro.tolist() == [0, 3, 3, 4, 4]
    assert dst.tolist() == [5, 8, 7, 0]


def _random_graph(rng, n, max_deg):
    rows = []
    for u in range(n):
        d = int(rng.integers(0, max_deg + 1)) if rng.random() < 0.7 else 0
        rows.append(list(rng.choice(n, size=min(d, n), replace=False)))
    return f.csr_from_rows(rows)


def test_expand_matches_loop():
    rng = np.random.default_rng(3)
    ro, dst = _random_graph(rng, 300, 12)
    for frontier in ([], [5], [7, 7, 7], list(rng.integers(0, 300, 500)), [299, 300, 10 ** 6, 0]):
        t, s = f.expand(ro, dst, np.asarray(frontier, dtype=np.int64))
        tl, sl = f.expand_loop(ro, dst, frontier)
        assert np.array_equal(t, tl) and np.array_equal(s, sl)


def test_power_law_graph_shape():
    ro, dst = power_law_graph(20000, 10.0, seed=5, max_deg=4096)
    n = len(ro) - 1
    deg = np.diff(ro.astype(np.int64))
    assert deg.max() <= 4096 and deg.min() >= 0 and 3 < deg.mean() < 30
    for u in list(np.argsort(-deg)[:20]) + list(range(0, n, 997)):
        row = dst[ro[u]:ro[u + 1]]
        assert len(set(row.tolist())) == len(row)          # one dictionary key per follower
        assert (row != u).all()                             # nobody follows themselves


def test_cascade_small_by_hand():
    tc = o.grain_type_code(f.CHIRPER_ACCOUNT_CLASS)
    # 0 -> {1, 2}, 1 -> {2, 3}, 2 -> {0}, 3 -> {4}, 4 -> {}
    ro, dst = f.csr_from_rows([[1, 2], [2, 3], [0], [4], []])
    silos = o.bench_silos(4)
    spec = o.ring_spec(silos, "D")
    reg = o.grain_keys(tc, np.arange(5))
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1]))
    d = o.DirectoryArrays(reg, np.arange(5), owner)
    hops = f.cascade(ro, dst, [0], 4, spec, d, 5, tc)
    assert hops[0]["target"].tolist() == [1, 2] and hops[0]["sender"].tolist() == [0, 0]
    assert hops[1]["frontier"].tolist() == [1, 2]
    assert hops[1]["target"].tolist() == [2, 3, 0] and hops[1]["sender"].tolist() == [1, 1, 2]
    # 0 was a seed and 2 already published: only 3 is new
    assert hops[2]["frontier"].tolist() == [3]
    assert hops[2]["target"].tolist() == [4]
    assert hops[3]["frontier"].tolist() == [4] and hops[3]["target"].size == 0
    assert (hops[1]["status"] == o.ST_OK).all()
    assert hops[1]["act"].tolist() == [2, 3, 0]
    assert hops[1]["perm"].tolist() == [2, 0, 1]


def test_partition_graph_rows():
    """partition_graph_np / _torch (the partitioned follower graph of gd_fanout_multi_part_device):
    local row i is node nodes[i]'s follower list, in enumeration order; the parts of all ranks hold
    every edge exactly once."""
    import torch
    from orleans_amd.fanout import partition_graph_np, partition_graph_torch
    from orleans_amd.workloads import power_law_graph
    n, W = 5000, 4
    ro, dst = power_law_graph(n, 5.0, seed=3, max_deg=300)
    owner = np.random.default_rng(1).integers(0, W, n)
    total = 0
    for r in range(W):
        nodes = np.nonzero(owner == r)[0]
        ro_l, dst_l, node_of = partition_graph_np(ro, dst, nodes)
        assert node_of.tolist() == nodes.tolist()
        for i in range(0, nodes.size, 37):
            u = nodes[i]
            assert dst_l[ro_l[i]:ro_l[i + 1]].tolist() == dst[ro[u]:ro[u + 1]].tolist()
        t_ro, t_dst, t_no = partition_graph_torch(torch.from_numpy(ro.astype(np.int64)),
                                                  torch.from_numpy(dst.astype(np.int32)),
                                                  torch.from_numpy(nodes.astype(np.int32)))
        assert t_ro.numpy().astype(np.uint32).tolist() == ro_l.tolist()
        assert t_dst.numpy().astype(np.uint32).tolist() == dst_l.tolist()
        assert t_no.numpy().tolist() == nodes.tolist()
        total += dst_l.size
    assert total == dst.size
