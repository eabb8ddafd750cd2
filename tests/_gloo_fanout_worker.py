"""Worker for tests/test_sharded_gloo.py::test_sharded_fanout_gloo: run under
`torch.distributed.run --nproc-per-node N` with the gloo backend on CPU.

Drives orleans_amd.fanout.ShardedFanout -- the exchange code the multi-GPU fan-out runs
over RCCL -- with a CPU engine built from the oracle (test infrastructure standing in for
DeviceFanoutEngine), and checks every hop against the single-node oracle cascade."""
import contextlib
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import fanout as fo                                  # noqa: E402
import oracle as o                                   # noqa: E402
from orleans_amd.fanout import ShardedFanout         # noqa: E402
from orleans_amd.workloads import power_law_graph     # noqa: E402

TC = o.grain_type_code(fo.CHIRPER_ACCOUNT_CLASS)
SPEC = o.ring_spec(o.bench_silos(8), "D")
N_NODES = 4000
HOPS = 4


def graph():
    return power_law_graph(N_NODES, 5.0, seed=77, max_deg=800)


def owners():
    reg = o.grain_keys(TC, np.arange(N_NODES))
    return o.ring_owner_np(SPEC, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)


def registered():
    return np.arange(N_NODES)[np.arange(N_NODES) % 17 != 5]      # some grains have no activation


class OracleFanoutEngine:
    """CPU stand-in for orleans_amd.fanout.DeviceFanoutEngine (same method contract)."""

    def __init__(self, rank, world):
        reg_nodes = registered()
        own = owners()[reg_nodes]
        mine = reg_nodes[own % world == rank]
        reg = o.grain_keys(TC, mine)
        self.dir = o.DirectoryArrays(reg, mine.astype(np.uint32), owners()[mine])

    @staticmethod
    def _t(a):
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32).copy())

    @staticmethod
    def _n(t):
        return t.numpy().view(np.uint32)

    def context(self):
        return contextlib.nullcontext()

    def expand(self, graph, frontier):
        t, s = fo.expand(graph[0], graph[1], self._n(frontier))
        return self._t(t), self._t(s)

    def pack_nodes_by_shard(self, nodes, payload, n_shards):
        nd = self._n(nodes)
        owner = o.ring_owner_np(SPEC, o.jenkins_u64x3_np(o.grain_keys(TC, nd.astype(np.int64))[:, 2],
                                                         np.zeros(nd.size, np.uint64), nd.astype(np.uint64)))
        perm, off = o.bucket_stable((owner % n_shards).astype(np.uint32), n_shards)
        counts = np.diff(off[:n_shards + 1]).astype(np.int32)
        return self._t(nd[perm]), self._t(self._n(payload)[perm]), torch.from_numpy(counts)

    def route_nodes_bucket(self, nodes, n_act):
        st, silo, act, _, _ = o.route_batch_np(o.grain_keys(TC, self._n(nodes).astype(np.int64)), SPEC, self.dir)
        perm, off = o.bucket_stable(act, n_act)
        return torch.from_numpy(st), self._t(silo), self._t(act), self._t(perm), self._t(off)

    def new_visited(self, n_act):
        return np.zeros(n_act, dtype=bool)

    def mark_visited(self, visited, nodes):
        nd = self._n(nodes)
        visited[nd[nd < visited.size]] = True

    def frontier_next(self, offsets, n_act, visited):
        return self._t(fo.next_frontier(self._n(offsets), n_act, visited))


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    ro, dst = graph()
    eng = OracleFanoutEngine(rank, world)
    seeds = np.random.default_rng(78).integers(0, N_NODES, 12).astype(np.uint32)
    hops = ShardedFanout(eng, (ro, dst), N_NODES).run(eng._t(seeds), HOPS)

    reg_nodes = registered()
    full = o.DirectoryArrays(o.grain_keys(TC, reg_nodes), reg_nodes.astype(np.uint32), owners()[reg_nodes])
    want = fo.cascade(ro, dst, seeds, HOPS, SPEC, full, N_NODES, TC)
    own_rank = owners() % world
    for h, (hr, wh) in enumerate(zip(hops, want)):
        fr = eng._n(hr.frontier)
        fronts = [None] * world
        dist.all_gather_object(fronts, fr.tolist())
        if h == 0:
            # each rank publishes the seeds it owns, in seed order
            for r in range(world):
                assert fronts[r] == [int(x) for x in seeds if own_rank[x] == r]
        else:
            # the union of the ranks' frontiers is the single-node frontier; each is owner-local
            assert sorted(sum(fronts, [])) == wh["frontier"].tolist(), h
            assert all(own_rank[x] == rank for x in fr)
        # arrival order here: sender rank by sender rank, each in that rank's emission order
        tt, ss = [], []
        for r in range(world):
            t, s = fo.expand(ro, dst, np.asarray(fronts[r], dtype=np.uint32))
            keep = own_rank[t] == rank
            tt.append(t[keep]); ss.append(s[keep])
        t, s = np.concatenate(tt), np.concatenate(ss)
        assert np.array_equal(eng._n(hr.target), t) and np.array_equal(eng._n(hr.sender), s), h
        st, silo, act, _, _ = o.route_batch_np(o.grain_keys(TC, t.astype(np.int64)), SPEC, full)
        assert np.array_equal(hr.status.numpy(), st)
        assert np.array_equal(eng._n(hr.act), act) and np.array_equal(eng._n(hr.silo), silo)
        wp, wo = o.bucket_stable(act, N_NODES)
        assert np.array_equal(eng._n(hr.perm), wp) and np.array_equal(eng._n(hr.offsets), wo)
        tot = torch.tensor([t.size], dtype=torch.int64)
        dist.all_reduce(tot)
        assert tot.item() == wh["target"].size, (h, tot.item(), wh["target"].size)
    print(f"OK fanout rank {rank}/{world}: {[eng._n(h.target).size for h in hops]} messages per hop", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
