"""Worker for tests/test_sharded_gloo.py::test_partitioned_fanout_gloo: run under
`torch.distributed.run --nproc-per-node N` with the gloo backend on CPU.

The partitioned fan-out cascade's host logic on CPU, the way gd_fanout_multi_part_device runs it on
the GPU: every rank keeps only the follower-graph rows of the grains it owns
(orleans_amd.fanout.partition_graph_np; partition_graph_torch must agree), resolves the seeds it
owns to its local rows in seed order, and per hop expands its publishers' rows, sends each
(target, sender) pair to the target's owner rank (torch.distributed all_to_all over gloo, the same
exchange the library does with grouped RCCL send/recv), routes + buckets what it receives
(oracle: test infrastructure standing in for the kernels), and takes its next publishers from its own
buckets.  Every hop must equal the replicated-graph oracle cascade (oracle/fanout.py cascade):
frontier, arrival order (sending rank, then emission order), routes and per-activation order.
Reference: Samples/Chirper/ChirperGrains/ChirperAccount.cs:106-147 (publish loop :131-134)."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import fanout as fo                                               # noqa: E402
import oracle as o                                                # noqa: E402
from orleans_amd.fanout import partition_graph_np, partition_graph_torch   # noqa: E402
from orleans_amd.workloads import power_law_graph                 # noqa: E402

TC = o.grain_type_code(fo.CHIRPER_ACCOUNT_CLASS)
N, HOPS = 3000, 4


def owners(spec, nodes):
    reg = o.grain_keys(TC, np.asarray(nodes, dtype=np.int64))
    return o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)


def exchange(parts):
    """all_to_all of one u32 array per peer (counts first): the concatenation by sending rank."""
    world = len(parts)
    sc = torch.tensor([p.size for p in parts], dtype=torch.int64)
    rc = torch.empty(world, dtype=torch.int64)
    dist.all_to_all_single(rc, sc)
    send = torch.from_numpy(np.concatenate(parts).astype(np.int64))
    recv = torch.empty(int(rc.sum()), dtype=torch.int64)
    dist.all_to_all_single(recv, send, output_split_sizes=rc.tolist(), input_split_sizes=sc.tolist())
    return recv.numpy().astype(np.uint32), rc.numpy()


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    ro, dst = power_law_graph(N, 5.0, seed=61, max_deg=400)
    own = owners(spec, np.arange(N))
    own_rank = own % world
    registered = np.arange(N)[np.arange(N) % 17 != 3]               # some followers have no activation
    mine = registered[own_rank[registered] == rank]                  # ascending node ids
    ro_l, dst_l, node_of = partition_graph_np(ro, dst, mine)
    t_ro, t_dst, t_no = partition_graph_torch(torch.from_numpy(ro.astype(np.int64)),
                                              torch.from_numpy(dst.astype(np.int32)),
                                              torch.from_numpy(mine.astype(np.int32)))
    assert np.array_equal(t_ro.numpy().view(np.uint32), ro_l)
    assert np.array_equal(t_dst.numpy().view(np.uint32), dst_l)
    assert np.array_equal(t_no.numpy().view(np.uint32), node_of)
    for i, u in enumerate(mine):                                     # row i = node mine[i]'s followers
        assert dst_l[ro_l[i]:ro_l[i + 1]].tolist() == dst[ro[u]:ro[u + 1]].tolist()
    n_rows = mine.size
    local = o.DirectoryArrays(o.grain_keys(TC, mine), np.arange(n_rows, dtype=np.uint32), own[mine])
    full = o.DirectoryArrays(o.grain_keys(TC, registered), registered.astype(np.uint32), own[registered])

    seeds = np.random.default_rng(4).choice(registered, 30).astype(np.uint32)
    seeds = np.concatenate([seeds, seeds[:2]]).astype(np.uint32)    # duplicates publish twice
    # hop 0: the seeds this rank owns, in seed order, resolved to local rows by the directory probe
    my_seeds = seeds[own_rank[seeds] == rank]
    st, _, rows, _, _ = o.route_batch_np(o.grain_keys(TC, my_seeds.astype(np.int64)), spec, local, my_silo=rank)
    assert (st == o.ST_OK).all(), "every seed has a live activation on its owner"
    frontier = rows.astype(np.uint32)
    visited = np.zeros(n_rows, dtype=bool)
    visited[frontier] = True
    want = fo.cascade(ro, dst, seeds, HOPS, spec, full, N, TC)
    total = 0
    for h in range(HOPS):
        fr_nodes = node_of[frontier]
        every = [None] * world
        dist.all_gather_object(every, fr_nodes.tolist())
        if h == 0:
            assert fr_nodes.tolist() == my_seeds.tolist()
        else:
            assert sorted(sum(every, [])) == want[h]["frontier"].tolist(), h
            assert (np.diff(fr_nodes.astype(np.int64)) > 0).all()
        # expand this rank's rows (senders as node ids), stable partition by the target's owner rank
        target, srow = fo.expand(ro_l, dst_l, frontier)
        sender = node_of[srow] if srow.size else srow
        dest = own_rank[target]
        t_recv, rc = exchange([target[dest == q] for q in range(world)])
        s_recv, _ = exchange([sender[dest == q] for q in range(world)])
        # arrival order: by sending rank, each rank's emission order (the replicated expansion of
        # each rank's publishers, filtered to this owner)
        tt, ss = [], []
        for q in range(world):
            t, s = fo.expand(ro, dst, np.asarray(every[q], dtype=np.uint32))
            keep = own_rank[t] == rank
            tt.append(t[keep]), ss.append(s[keep])
        assert t_recv.tolist() == np.concatenate(tt).tolist(), (h, "target")
        assert s_recv.tolist() == np.concatenate(ss).tolist(), (h, "sender")
        keys = o.grain_keys(TC, t_recv.astype(np.int64))
        st, silo, act, _, _ = o.route_batch_np(keys, spec, local, my_silo=rank)
        st_f, silo_f, act_f, _, _ = o.route_batch_np(keys, spec, full, my_silo=rank)
        assert np.array_equal(st, st_f) and np.array_equal(silo, silo_f), h
        ok = st == o.ST_OK
        assert np.array_equal(node_of[act[ok]], act_f[ok]), h
        perm, off = o.bucket_stable(act, n_rows)
        pf, of = o.bucket_stable(act_f, N)
        for i, u in enumerate(node_of):                              # each activation's messages, in order
            assert perm[off[i]:off[i + 1]].tolist() == pf[of[u]:of[u + 1]].tolist(), (h, i)
        total += int(t_recv.size)
        frontier = fo.next_frontier(off, n_rows, visited)
    all_total = torch.tensor([total], dtype=torch.int64)
    dist.all_reduce(all_total)
    assert int(all_total.item()) == sum(w["target"].size for w in want)
    assert int(all_total.item()) > 1000
    print(f"OK rank {rank}/{world} partitioned fan-out ({total} messages received)", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
