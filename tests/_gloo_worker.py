"""Worker for tests/test_sharded_gloo.py: run under
`torch.distributed.run --nproc-per-node N` with the gloo backend on CPU.

It drives orleans_amd.sharded.ShardedRouter -- the exact exchange code bench.py
runs over RCCL -- with a CPU engine built from the oracle (test infrastructure
standing in for the GPU engine), and checks the sharded results against a
single-node oracle run."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as o                                   # noqa: E402
from orleans_amd.sharded import ShardedRouter        # noqa: E402

TC = o.grain_type_code(o.PING_GRAIN_CLASS)
SPEC = o.ring_spec(o.bench_silos(8), "D")
G_TOTAL = 3000
N_PER_RANK = 20000


def batch_of(rank):
    rng = np.random.default_rng(1000 + rank)
    keys = o.grain_keys(TC, rng.integers(0, G_TOTAL + 200, size=N_PER_RANK))   # ~6% unregistered
    keys[::997] = np.array(o.UniqueKey(0, 7, o.type_code_data(o.CAT_SYSTEM_TARGET, 1)).as_tuple(), dtype=np.uint64)
    return keys


class OracleEngine:
    """CPU stand-in for orleans_amd.sharded.DeviceEngine (same method contract)."""

    def __init__(self, rank, world, my_silo):
        self.rank, self.world, self.my_silo = rank, world, my_silo
        reg = o.grain_keys(TC, np.arange(G_TOTAL))
        own = o.ring_owner_np(SPEC, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1]))
        mine = np.nonzero(own % world == rank)[0]
        self.n_act = len(mine)
        self.dir = o.DirectoryArrays(reg[mine], np.arange(self.n_act), own[mine])
        self.local_act_of_grain = {int(g): i for i, g in enumerate(mine)}
        self.spec = SPEC

    def pack_by_shard(self, keys, n_shards):
        k = keys.numpy().view(np.uint64)
        st, silo, act, owner, h = o.route_batch_np(k, self.spec,
                                                   o.DirectoryArrays(np.zeros((0, 3), np.uint64), [], []),
                                                   my_silo=self.my_silo, seed_silo=0)
        owner = np.where(owner == o.M32, self.my_silo, owner)
        dest = (owner % n_shards).astype(np.uint32)
        perm, off = o.bucket_stable(dest, n_shards)
        counts = np.diff(off[: n_shards + 1]).astype(np.int32)
        return (torch.from_numpy(k[perm].view(np.int64).copy()), torch.from_numpy(perm.astype(np.int32)),
                torch.from_numpy(counts))

    def route_bucket(self, keys, n_act):
        k = keys.numpy().view(np.uint64)
        st, silo, act, owner, h = o.route_batch_np(k, SPEC, self.dir, my_silo=self.my_silo, seed_silo=0)
        perm, off = o.bucket_stable(act, n_act)
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt))
        return (t(st, np.uint8), t(silo, np.int32), t(act, np.int32), t(perm, np.int32), t(off, np.int32))


    def route(self, keys):
        k = keys.numpy().view(np.uint64)
        st, silo, act, _, _ = o.route_batch_np(k, self.spec, self.dir, my_silo=self.my_silo, seed_silo=0)
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).view(dt))
        return t(st, np.uint8), t(silo, np.int32), t(act, np.int32)

    def bucket(self, act, n_act):
        perm, off = o.bucket_stable(act.numpy().view(np.uint32), n_act)
        return torch.from_numpy(perm.view(np.int32)), torch.from_numpy(off.view(np.int32))

    def pack_routes_by_rank(self, keys, st, silo, n_shards, my_rank):
        s, sl = st.numpy(), silo.numpy().view(np.uint32)
        dest = np.where(s == o.ST_OK, sl % n_shards, my_rank).astype(np.uint32)
        perm, off = o.bucket_stable(dest, n_shards)
        counts = np.diff(off[: n_shards + 1]).astype(np.int32)
        k = keys.numpy()
        return torch.from_numpy(k[perm].copy()), torch.from_numpy(perm.astype(np.int32)), torch.from_numpy(counts)


class ForwardEngine(OracleEngine):
    """Activations not co-located with their directory owner: grain g lives on silo (5g + 1) % 8,
    activation id = its index among the grains hosted on that silo's rank."""

    def __init__(self, rank, world, my_silo):
        super().__init__(rank, world, my_silo)
        reg = o.grain_keys(TC, np.arange(G_TOTAL))
        own = o.ring_owner_np(SPEC, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1]))
        act_silo = ((5 * np.arange(G_TOTAL) + 1) % 8).astype(np.uint32)
        host = act_silo % world
        act_id = np.zeros(G_TOTAL, np.uint32)
        for r in range(world):
            act_id[host == r] = np.arange(int((host == r).sum()))
        self.n_act = int((host == rank).sum())
        mine = own % world == rank
        self.dir = o.DirectoryArrays(reg[mine], act_id[mine], act_silo[mine])
        self.full = o.DirectoryArrays(reg, act_id, act_silo)


def check_forward(rank, world):
    """ShardedRouter.route_bucket(forward=True): every message ends on the rank hosting its
    activation (directory hits) or on its owner (anything else), with the owner's route, and each
    activation's messages in (sender rank, sender batch order)."""
    eng = ForwardEngine(rank, world, my_silo=rank)
    router = ShardedRouter(eng)
    keys = torch.from_numpy(batch_of(rank).view(np.int64).copy())
    res = router.route_bucket(keys, eng.n_act, forward=True)
    rk = res.recv_keys.numpy().view(np.uint64)
    src, idx = res.recv_src.numpy(), res.recv_idx.numpy()
    batches = {r: batch_of(r) for r in range(world)}
    expect = []
    for r in range(world):
        st, silo, act, owner, _ = o.route_batch_np(batches[r], SPEC, eng.full, my_silo=r, seed_silo=0)
        orank = np.where(owner == o.M32, r, owner % world)
        final = np.where(st == o.ST_OK, silo % world, orank)
        for i in np.nonzero(final == rank)[0]:
            expect.append((int(orank[i]), r, int(i)))
    # arrival order = (owner rank, sender rank, sender order)
    expect.sort()
    assert [(s_, i_) for _, s_, i_ in expect] == list(zip(src.tolist(), idx.tolist()))
    for j in range(len(rk)):
        assert (batches[src[j]][idx[j]] == rk[j]).all()
    # the owner's routes (a system target's owner is its sender's silo, which is this rank)
    w_st, w_silo, w_act, _, _ = o.route_batch_np(rk, SPEC, eng.full, my_silo=rank, seed_silo=0)
    assert np.array_equal(res.status.numpy(), w_st)
    assert np.array_equal(res.silo.numpy().view(np.uint32), w_silo)
    assert np.array_equal(res.act.numpy().view(np.uint32), w_act)
    ok = w_st == o.ST_OK
    assert (w_silo[ok] % world == rank).all()
    wp, wo = o.bucket_stable(res.act.numpy().view(np.uint32), eng.n_act)
    assert np.array_equal(res.perm.numpy().view(np.uint32), wp)
    assert np.array_equal(res.offsets.numpy().view(np.uint32), wo)
    # per activation: (sender rank, sender order) increasing
    order = src.astype(np.int64) * (1 << 32) + idx
    perm = wp
    for a in range(eng.n_act):
        seg = order[perm[wo[a]:wo[a + 1]]]
        assert (np.diff(seg) > 0).all()
    tot = torch.tensor([len(rk), int(ok.sum())], dtype=torch.int64)
    dist.all_reduce(tot)
    assert tot[0].item() == world * N_PER_RANK
    return int(ok.sum())


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    eng = OracleEngine(rank, world, my_silo=rank)
    router = ShardedRouter(eng)
    keys = torch.from_numpy(batch_of(rank).view(np.int64).copy())
    res = router.route_bucket(keys, eng.n_act)
    m = res.recv_keys.shape[0]
    rk = res.recv_keys.numpy().view(np.uint64)
    src = res.recv_src.numpy()
    idx = res.recv_idx.numpy()
    # 1) every received header is the sender's message at (src, idx)
    batches = {r: batch_of(r) for r in range(world)}
    for j in range(m):
        assert (batches[src[j]][idx[j]] == rk[j]).all()
    # 2) arrival order: grouped by sender rank, each group in the sender's batch order
    order = src.astype(np.int64) * (1 << 32) + idx
    assert (np.diff(order) > 0).all()
    # 3) this rank owns what it received (system targets stay with their sender's silo)
    st, silo, act, owner, h = o.route_batch_np(rk, SPEC, eng.dir, my_silo=rank, seed_silo=0)
    owner = np.where(owner == o.M32, src, owner)
    is_sys = st == o.ST_SYSTEM_TARGET
    assert ((owner[~is_sys] % world) == rank).all()
    # 4) routed results = the oracle on the received headers; per-activation FIFO
    assert np.array_equal(res.status.numpy(), st)
    assert np.array_equal(res.act.numpy().view(np.uint32), act)
    wp, wo = o.bucket_stable(act, eng.n_act)
    assert np.array_equal(res.perm.numpy().view(np.uint32), wp)
    assert np.array_equal(res.offsets.numpy().view(np.uint32), wo)
    # 5) nothing lost: messages received over all ranks == messages sent
    tot = torch.tensor([m], dtype=torch.int64)
    dist.all_reduce(tot)
    assert tot.item() == world * N_PER_RANK
    # 6) every OK message found its grain: act is the owner's local index of that grain
    ok = st == o.ST_OK
    assert (rk[ok, 1] < G_TOTAL).all()
    for j in np.nonzero(ok)[0][:500]:
        assert act[j] == eng.local_act_of_grain[int(rk[j, 1])]
    # 7) activations away from their directory owner: the forward hop (SURVEY 8 e caveat)
    n_fwd_ok = check_forward(rank, world)
    # (the multi-rank directory handoff is the library's gd_dir_handoff_multi, GPU-tested at W = 8
    # against oracle/dirstate.py in tests/test_gpu_handoff_multi.py)
    print(f"OK rank {rank}/{world}: received {m}, ok {int(ok.sum())}, forwarded-ok {n_fwd_ok}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
