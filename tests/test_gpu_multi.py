"""In-library exchange over RCCL (gd_comm_* + gd_route_multi*, SURVEY 8 b / 8 e) against the
oracle: the sender's batch is partitioned by owner rank (OutboundMessageQueue.cs:54-131 per
target silo), exchanged, probed and bucketed on the owner (GrainDirectoryPartition.cs:385-441,
ActivationData.cs:566-606), and the routes come back in the sender's batch order
(Dispatcher.AddressMessage, Dispatcher.cs:715-767).  World 1 runs the whole path (the exchange
is a send/recv to self); the 2-rank case runs two processes on cuda:0 if RCCL allows it."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle as o

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TC = o.grain_type_code(o.PING_GRAIN_CLASS)


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


def _directory(G, world, rank, spec):
    reg = o.grain_keys(TC, np.arange(G))
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    mine = np.nonzero(own % world == rank)[0]
    return reg, own, mine


@pytest.mark.parametrize("n", [0, 1, 4999, 100003])
def test_route_multi_world1(gd, n):
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    G = 4096
    reg, own, mine = _directory(G, 1, 0, spec)
    rng = np.random.default_rng(n + 11)
    keys = o.grain_keys(TC, rng.integers(0, G + 300, size=n))
    if n > 100:
        keys[::13] = np.array(o.UniqueKey(0, 7, o.type_code_data(o.CAT_SYSTEM_TARGET, 1)).as_tuple(), dtype=np.uint64)
    e = gd.GrainDispatch(device=0, table_capacity=1 << 14, my_silo=2)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    e.register(reg, np.arange(G), own)
    e.comm_init(gd.GrainDispatch.comm_unique_id(), 1, 0)
    ro = o.region_order(keys)              # arrival order: by table region, batch order within one
    for ret in (False, True):
        r = e.route_multi(keys, G, return_routes=ret)
        st, silo, act, _, _ = o.route_batch_np(keys, spec, o.DirectoryArrays(reg, np.arange(G), own), my_silo=2)
        np.testing.assert_array_equal(r["recv_keys"], keys[ro])
        np.testing.assert_array_equal(r["recv_idx"], ro.astype(np.uint32))
        np.testing.assert_array_equal(r["recv_src"], np.zeros(n, np.uint32))
        np.testing.assert_array_equal(r["status"], st[ro])
        np.testing.assert_array_equal(r["silo"], silo[ro])
        np.testing.assert_array_equal(r["act"], act[ro])
        wp, wo = o.bucket_stable(act[ro], G)
        np.testing.assert_array_equal(r["perm"], wp)
        np.testing.assert_array_equal(r["offsets"], wo)
        if ret:                            # back in the sender's batch order
            np.testing.assert_array_equal(r["ret_status"], st)
            np.testing.assert_array_equal(r["ret_silo"], silo)
            np.testing.assert_array_equal(r["ret_act"], act)
    e.comm_destroy()
    with pytest.raises(gd.GrainDispatchError):
        e.route_multi(keys, G)              # no communicator any more: GD_ESTATE
    e.close()


def test_route_multi_device_pointers(gd):
    """gd_route_multi_device on torch-allocated HBM keys; results read through the returned
    device pointers (library-owned buffers)."""
    import torch
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "V")
    G, n = 2048, 30000
    e = gd.GrainDispatch(device=0, table_capacity=1 << 13)
    e.ring_set_silos("V", [(s.ip, s.port, s.gen) for s in silos])
    reg, own, _ = _directory(G, 1, 0, spec)
    e.register(reg, np.arange(G), own)
    e.comm_init(gd.GrainDispatch.comm_unique_id(), 1, 0)
    keys = o.grain_keys(TC, np.random.default_rng(3).integers(0, G, size=n))
    tk = torch.from_numpy(keys.view(np.int64).copy()).cuda()
    stream = torch.cuda.Stream()
    e.set_stream(stream.cuda_stream)
    with torch.cuda.stream(stream):
        r = e.route_multi_device(tk.data_ptr(), n, G, return_routes=True)
    torch.cuda.synchronize()
    assert r.n_recv == n and r.ret_act and r.perm
    got = e.multi_fetch(r, n)
    st, silo, act, _, _ = o.route_batch_np(keys, spec, o.DirectoryArrays(reg, np.arange(G), own))
    ro = o.region_order(keys)
    np.testing.assert_array_equal(got["act"], act[ro])
    np.testing.assert_array_equal(got["ret_act"], act)
    np.testing.assert_array_equal(got["ret_silo"], silo)
    wp, wo = o.bucket_stable(act[ro], G)
    np.testing.assert_array_equal(got["perm"], wp)
    np.testing.assert_array_equal(got["offsets"], wo)
    e.comm_destroy()
    e.close()


def test_route_multi_two_ranks_one_gpu(tmp_path):
    """Two processes, one communicator, both on cuda:0.  Skips if RCCL refuses two ranks on one
    device; the 8-GPU form runs in bench.py --exchange library."""
    world, n = 2, 20011
    env = dict(os.environ)
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_rccl_worker.py"), str(tmp_path),
                               str(world), str(r), str(n)], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("RCCL worker timed out")
        outs.append(out)
    codes = [p.returncode for p in procs]
    if 77 in codes:
        pytest.skip("RCCL refuses two ranks on one GPU: " + " | ".join(x.strip()[-300:] for x in outs))
    assert codes == [0] * world, outs
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _rccl_worker as w
    spec = o.ring_spec(o.bench_silos(8), "D")
    reg, own, _ = _directory(w.G_TOTAL, 1, 0, spec)
    res = [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)]
    batches = [w.batch_of(r, n) for r in range(world)]
    for r in range(world):
        mine = np.nonzero(own % world == r)[0]
        local = np.full(w.G_TOTAL, o.M32, np.int64)
        local[mine] = np.arange(len(mine))
        d = o.DirectoryArrays(reg[mine], np.arange(len(mine)), own[mine])
        exp_keys, exp_idx, exp_src = [], [], []
        for s in range(world):
            k = batches[s]
            _, _, _, owner, _ = o.route_batch_np(k, spec, o.DirectoryArrays(np.zeros((0, 3), np.uint64), [], []))
            sel = np.nonzero(owner % world == r)[0]
            sel = sel[o.region_order(k[sel])]
            exp_keys.append(k[sel]), exp_idx.append(sel), exp_src.append(np.full(len(sel), s))
        ek = np.concatenate(exp_keys)
        np.testing.assert_array_equal(res[r]["recv_keys"], ek)
        np.testing.assert_array_equal(res[r]["recv_idx"], np.concatenate(exp_idx))
        np.testing.assert_array_equal(res[r]["recv_src"], np.concatenate(exp_src))
        st, silo, act, _, _ = o.route_batch_np(ek, spec, d, my_silo=r)
        np.testing.assert_array_equal(res[r]["status"], st)
        np.testing.assert_array_equal(res[r]["act"], act)
        wp, wo = o.bucket_stable(act, len(mine))
        np.testing.assert_array_equal(res[r]["perm"], wp)
        np.testing.assert_array_equal(res[r]["offsets"], wo)
    # routes back at each sender, in batch order, equal the owner's answer
    for s in range(world):
        k = batches[s]
        _, _, _, owner, _ = o.route_batch_np(k, spec, o.DirectoryArrays(np.zeros((0, 3), np.uint64), [], []))
        for r in range(world):
            mine = np.nonzero(own % world == r)[0]
            d = o.DirectoryArrays(reg[mine], np.arange(len(mine)), own[mine])
            sel = np.nonzero(owner % world == r)[0]
            st, silo, act, _, _ = o.route_batch_np(k[sel], spec, d, my_silo=r)
            np.testing.assert_array_equal(res[s]["ret_status"][sel], st)
            np.testing.assert_array_equal(res[s]["ret_act"][sel], act)
            np.testing.assert_array_equal(res[s]["ret_silo"][sel], silo)


def test_route_multi_pipelined_batches(gd):
    """GD_MULTI_KEYS_READY: batch i+1's partition + exchange (library exchange stream) overlap
    batch i's probe + bucketing (handle stream); results of a batch stay valid through the next
    call.  Five different batches, each checked after the call that follows it."""
    import torch
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    G = 50000
    e = gd.GrainDispatch(device=0, table_capacity=1 << 17, my_silo=1)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    reg, own, _ = _directory(G, 1, 0, spec)
    e.register(reg, np.arange(G), own)
    e.comm_init(gd.GrainDispatch.comm_unique_id(), 1, 0)
    stream = torch.cuda.Stream()
    e.set_stream(stream.cuda_stream)
    d = o.DirectoryArrays(reg, np.arange(G), own)
    batches = [o.grain_keys(TC, np.random.default_rng(40 + i).integers(0, G + 500, size=200000 + 7919 * i))
               for i in range(5)]
    dev_keys = [torch.from_numpy(b.view(np.int64).copy()).cuda() for b in batches]
    torch.cuda.synchronize()
    prev = None
    for i in range(len(batches) + 1):
        if i < len(batches):
            with torch.cuda.stream(stream):
                r = e.route_multi_device(dev_keys[i].data_ptr(), len(batches[i]), G, return_routes=(i % 2 == 1),
                                         keys_ready=True)
            cur = (i, r)
        if prev is not None:
            j, rp = prev
            e.synchronize()
            m = rp.n_recv
            assert m == len(batches[j])
            act = torch.as_tensor(_Cai(rp.act, m), device="cuda").cpu().numpy().view(np.uint32)
            perm = torch.as_tensor(_Cai(rp.perm, m), device="cuda").cpu().numpy().view(np.uint32)
            offs = torch.as_tensor(_Cai(rp.offsets, G + 2), device="cuda").cpu().numpy().view(np.uint32)
            st, silo, want_act, _, _ = o.route_batch_np(batches[j], spec, d, my_silo=1)
            ro = o.region_order(batches[j])
            np.testing.assert_array_equal(act, want_act[ro])
            wp, wo = o.bucket_stable(want_act[ro], G)
            np.testing.assert_array_equal(perm, wp)
            np.testing.assert_array_equal(offs, wo)
            if j % 2 == 1:
                ra = torch.as_tensor(_Cai(rp.ret_act, m), device="cuda").cpu().numpy().view(np.uint32)
                np.testing.assert_array_equal(ra, want_act)
        prev = cur if i < len(batches) else None
    e.comm_destroy()
    e.close()


class _Cai:
    def __init__(self, ptr, n, typestr="<i4"):
        shape = n if isinstance(n, tuple) else (n,)
        self.__cuda_array_interface__ = {"shape": shape, "typestr": typestr, "data": (int(ptr), False), "version": 3,
                                         "strides": None}


@pytest.mark.parametrize("n", [0, 7, 30011])
def test_route_multi_ext_world1(gd, n):
    """gd_route_multi_ext: KeyExt grains partitioned by their KeyExt hash, strings carried in the
    byte round, routed on the owner; results and returned routes against oracle/keyext.py."""
    import keyext as kx
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    G = 2048
    reg, own, _ = _directory(G, 1, 0, spec)
    e = gd.GrainDispatch(device=0, table_capacity=1 << 13, my_silo=4)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    e.register(reg, np.arange(G), own)
    stc = o.grain_type_code("UnitTests.GrainInterfaces.IStringKeyGrain")
    names = [f"acct:{i}" + "ß" * (i % 4) + "z" * (i % 50) for i in range(400)]
    tcd = o.type_code_data(o.CAT_KEYEXT_GRAIN, stc)
    d = kx.KeyExtDirectory()
    e.register_ext(np.tile(np.array([[0, 0, tcd]], np.uint64), (200, 1)), names[:200], np.arange(200) + G,
                   np.arange(200) % 8)
    for i in range(200):
        d.add_single_activation((0, 0, tcd), names[i].encode(), G + i, i % 8)
    rng = np.random.default_rng(n + 3)
    keys = o.grain_keys(TC, rng.integers(0, G + 100, size=n))
    exts = [None] * n
    for i in np.nonzero(rng.random(n) < 0.4)[0]:
        keys[i] = (0, 0, tcd)
        exts[i] = names[int(rng.integers(0, 400))].encode()
    for i in range(0, n, 97):
        if exts[i] is not None:
            exts[i] = kx.EXT_HOST
    e.comm_init(gd.GrainDispatch.comm_unique_id(), 1, 0)
    bexts = [gd.GD_KEYEXT_HOST if (isinstance(x, str) and x == kx.EXT_HOST) else x for x in exts]
    r = e.route_multi_ext(keys, bexts, G + 200, return_routes=True)
    st, silo, act, _, _ = kx.route_batch_ext(keys, exts, spec, o.DirectoryArrays(reg, np.arange(G), own), d, my_silo=4)
    ro = o.region_order(keys)              # KeyExt grains: region 0
    np.testing.assert_array_equal(r["recv_keys"], keys[ro])
    np.testing.assert_array_equal(r["status"], st[ro])
    np.testing.assert_array_equal(r["silo"], silo[ro])
    np.testing.assert_array_equal(r["act"], act[ro])
    wp, wo = o.bucket_stable(act[ro], G + 200)
    np.testing.assert_array_equal(r["perm"], wp)
    np.testing.assert_array_equal(r["offsets"], wo)
    np.testing.assert_array_equal(r["ret_act"], act)
    np.testing.assert_array_equal(r["ret_status"], st)
    if n > 1000:
        assert ((st == o.ST_OK) & (keys[:, 2] == np.uint64(tcd))).sum() > n // 10
    e.comm_destroy()
    e.close()


@pytest.mark.parametrize("mode", ["D", "R", "V"])
def test_ring_owner_ext_is_the_partition_owner(gd, mode):
    """gd_ring_owner_ext runs the exchange partition's owner function (key_dest, gd_shard.h):
    KeyExt grains by their KeyExt hash, null KeyExt by the three words, GD_KEYEXT_HOST and system
    targets to my silo, the membership grain to the seed (LocalGrainDirectory.cs:477-545)."""
    import keyext as kx
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, mode)
    e = gd.GrainDispatch(device=0, table_capacity=1 << 10, my_silo=5, seed_silo=2)
    e.ring_set_silos(mode, [(s.ip, s.port, s.gen) for s in silos])
    rng = np.random.default_rng(9)
    n = 4000
    keys = o.grain_keys(TC, rng.integers(0, 10 ** 6, size=n))
    exts = [None] * n
    geo = o.type_code_data(o.CAT_GEO_CLIENT, 0)
    for i in range(n):
        c = i % 6
        if c == 1:
            keys[i] = (0, 0, o.type_code_data(o.CAT_KEYEXT_GRAIN, 77))
            exts[i] = ("k%d" % i + "é" * (i % 9) + "x" * (i % 70)).encode()
        elif c == 2:
            keys[i] = (i, 1, geo)                      # geo client with a null KeyExt
        elif c == 3:
            keys[i] = (0, 0, o.type_code_data(o.CAT_KEYEXT_GRAIN, 77))
            exts[i] = kx.EXT_HOST
    keys[5::97] = np.array(o.UniqueKey(0, 3, o.type_code_data(o.CAT_SYSTEM_TARGET, 1)).as_tuple(), dtype=np.uint64)
    keys[7::89] = np.array(o.MEMBERSHIP_TABLE_ID.as_tuple(), dtype=np.uint64)
    for i in list(range(5, n, 97)) + list(range(7, n, 89)):
        exts[i] = None
    bexts = [gd.GD_KEYEXT_HOST if (isinstance(x, str) and x == kx.EXT_HOST) else x for x in exts]
    got = e.ring_owner_ext(keys, bexts)
    _, _, _, owner, _ = kx.route_batch_ext(keys, exts, spec, o.DirectoryArrays(np.zeros((0, 3), np.uint64), [], []),
                                           kx.KeyExtDirectory(), my_silo=5, seed_silo=2)
    want = np.where(owner == o.M32, 5, owner)          # KEYEXT kept here -> my silo
    np.testing.assert_array_equal(got, want)
    e.close()


@pytest.mark.parametrize("n,mixed", [(0, False), (1, False), (70001, False), (70001, True)])
def test_route_multi_forward_world1(gd, n, mixed):
    """GD_MULTI_FORWARD at world 1: the forward hop is a send to self, so the result equals the
    co-located one (the activation silos here differ from the owners).  One grain type with small
    keys: the forward round moves u32 N1s (descriptor mode 2) and the keys are rebuilt; mixed
    (system targets among them): 24-B keys."""
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "R")
    G = 3000
    reg, own, _ = _directory(G, 1, 0, spec)
    act_silo = ((5 * np.arange(G) + 1) % 8).astype(np.uint32)
    rng = np.random.default_rng(n + 5)
    keys = o.grain_keys(TC, rng.integers(0, G + 200, size=n))
    if mixed:
        keys[::17] = np.array(o.UniqueKey(0, 7, o.type_code_data(o.CAT_SYSTEM_TARGET, 1)).as_tuple(), np.uint64)
    e = gd.GrainDispatch(device=0, table_capacity=1 << 13, my_silo=4)
    e.ring_set_silos("R", [(s.ip, s.port, s.gen) for s in silos])
    e.register(reg, np.arange(G), act_silo)
    e.comm_init(gd.GrainDispatch.comm_unique_id(), 1, 0)
    st, silo, act, _, _ = o.route_batch_np(keys, spec, o.DirectoryArrays(reg, np.arange(G), act_silo), my_silo=4)
    ro = o.region_order(keys)
    wp, wo = o.bucket_stable(act[ro], G)
    for ret in (False, True):
        r = e.route_multi(keys, G, return_routes=ret, forward=True)
        np.testing.assert_array_equal(r["recv_keys"], keys[ro])
        np.testing.assert_array_equal(r["recv_idx"], ro.astype(np.uint32))
        np.testing.assert_array_equal(r["recv_src"], np.zeros(n, np.uint32))
        np.testing.assert_array_equal(r["status"], st[ro])
        np.testing.assert_array_equal(r["silo"], silo[ro])
        np.testing.assert_array_equal(r["act"], act[ro])
        np.testing.assert_array_equal(r["perm"], wp)
        np.testing.assert_array_equal(r["offsets"], wo)
        if ret:
            np.testing.assert_array_equal(r["ret_act"], act)
    e.comm_destroy()
    e.close()


@pytest.mark.parametrize("W", [1, 2, 3, 8, 256])
def test_pack_routes_by_rank(gd, W):
    """gd_pack_routes_by_rank_device: stable partition by silo % W for directory hits, my_rank for
    every other status."""
    import torch
    rng = np.random.default_rng(W)
    for n in (0, 1, 2047, 2048, 2049, 300001):
        my_rank = int(rng.integers(0, W))
        keys = rng.integers(0, 1 << 62, size=(n, 3), dtype=np.uint64)
        st = rng.choice(np.array([0, 0, 0, 1, 2, 3, 4, 7], np.uint8), size=n)
        silo = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
        e = gd.GrainDispatch(device=0, table_capacity=64)
        dk = torch.from_numpy(keys.view(np.int64).copy()).cuda()
        ds = torch.from_numpy(st.copy()).cuda()
        dl = torch.from_numpy(silo.view(np.int32).copy()).cuda()
        sk = torch.empty_like(dk)
        sp = torch.empty(n, dtype=torch.int32, device="cuda")
        cnt = torch.empty(W, dtype=torch.int32, device="cuda")
        e.pack_routes_by_rank_device(dk.data_ptr(), ds.data_ptr(), dl.data_ptr(), n, W, my_rank, sk.data_ptr(),
                                     sp.data_ptr(), cnt.data_ptr())
        e.synchronize()
        dest = np.where(st == 0, silo % W, my_rank).astype(np.uint32)
        wp, wo = o.bucket_stable(dest, W)
        np.testing.assert_array_equal(sp.cpu().numpy().view(np.uint32), wp)
        np.testing.assert_array_equal(sk.cpu().numpy().view(np.uint64), keys[wp])
        np.testing.assert_array_equal(cnt.cpu().numpy(), np.diff(wo[:W + 1]))
        e.close()
    with pytest.raises(gd.GrainDispatchError):
        gd.GrainDispatch(device=0, table_capacity=64).pack_routes_by_rank_device(0, 0, 0, 0, W, W, 0, 0, 0)


def test_sharded_forward_two_ranks_one_gpu(tmp_path):
    """ShardedRouter.route_bucket(forward=True) with the device engine, two ranks on cuda:0 over
    gloo (host-staged): every message ends on the rank hosting its activation (directory hits) or
    on its owner (the rest), with the owner's route, and each activation sees its messages in
    (sender rank, sender batch order)."""
    world, n = 2, 30011
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_gpu_forward_worker.py"), str(tmp_path),
                               str(world), str(r), str(n)], cwd=ROOT, env=dict(os.environ), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(world)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=100)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            pytest.fail("forward worker timed out")
        outs.append(out)
    assert [p.returncode for p in procs] == [0] * world, outs
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import _gpu_forward_worker as w
    spec, reg, own, act_silo, act_id = w.directory(world)
    full = o.DirectoryArrays(reg, act_id, act_silo)
    batches = [w.batch_of(r, n) for r in range(world)]
    expect = {r: [] for r in range(world)}
    for s in range(world):
        st, silo, act, owner, _ = o.route_batch_np(batches[s], spec, full, my_silo=s)
        orank = np.where(owner == o.M32, s, owner % world)
        final = np.where(st == o.ST_OK, silo % world, orank)
        for i in range(n):
            expect[int(final[i])].append((int(orank[i]), s, i))
    for r in range(world):
        res = dict(np.load(tmp_path / f"fwd{r}.npz"))
        ex = sorted(expect[r])
        np.testing.assert_array_equal(res["recv_src"], np.array([x[1] for x in ex], np.uint32))
        np.testing.assert_array_equal(res["recv_idx"], np.array([x[2] for x in ex], np.uint32))
        rk = np.concatenate([batches[x[1]][x[2]:x[2] + 1] for x in ex]) if ex else np.zeros((0, 3), np.uint64)
        np.testing.assert_array_equal(res["recv_keys"], rk)
        st, silo, act, _, _ = o.route_batch_np(rk, spec, full, my_silo=r)
        np.testing.assert_array_equal(res["status"], st)
        np.testing.assert_array_equal(res["silo"], silo)
        np.testing.assert_array_equal(res["act"], act)
        n_act = int((act_silo % world == r).sum())
        wp, wo = o.bucket_stable(act, n_act)
        np.testing.assert_array_equal(res["perm"], wp)
        np.testing.assert_array_equal(res["offsets"], wo)
    # without the forward hop: everything stays on its owner (ShardedRouter.exchange + route_bucket)
    for r in range(world):
        res = dict(np.load(tmp_path / f"own{r}.npz"))
        ks, ids, srcs = [], [], []
        for s in range(world):
            _, _, _, owner, _ = o.route_batch_np(batches[s], spec, full, my_silo=s)
            sel = np.nonzero(np.where(owner == o.M32, s, owner % world) == r)[0]
            ks.append(batches[s][sel]), ids.append(sel), srcs.append(np.full(len(sel), s))
        rk = np.concatenate(ks)
        np.testing.assert_array_equal(res["recv_keys"], rk)
        np.testing.assert_array_equal(res["recv_idx"], np.concatenate(ids).astype(np.uint32))
        np.testing.assert_array_equal(res["recv_src"], np.concatenate(srcs).astype(np.uint32))
        st, silo, act, _, _ = o.route_batch_np(rk, spec, full, my_silo=r)
        np.testing.assert_array_equal(res["status"], st)
        np.testing.assert_array_equal(res["silo"], silo)
        np.testing.assert_array_equal(res["act"], act)
        wp, wo = o.bucket_stable(act, w.G_TOTAL)
        np.testing.assert_array_equal(res["perm"], wp)
        np.testing.assert_array_equal(res["offsets"], wo)


# ---- W > 1 in one process (gd_comm_init_local): the library exchange at several ranks ----------
def _run_ranks(fns):
    """Run fns[r]() on one thread per rank; re-raise the first failure."""
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


def _local_world(gd, W, spec_mode, silos, reg, act, silo_of, my_silos=None):
    """W engines on cuda:0, rank r holding the directory entries whose ring owner lives on r."""
    spec = o.ring_spec(silos, spec_mode)
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    es = []
    for r in range(W):
        e = gd.GrainDispatch(device=0, table_capacity=1 << 13, my_silo=r if my_silos is None else my_silos[r])
        e.ring_set_silos(spec_mode, [(s.ip, s.port, s.gen) for s in silos])
        mine = own % W == r
        e.register(reg[mine], act[mine], silo_of[mine])
        es.append(e)
    gd.GrainDispatch.comm_init_local(es)
    return spec, own, es


def _expected_owner_side(batches, spec, full, W, r, by_region=True):
    """Messages rank r owns, in arrival order (sender rank, table region, sender order), and their
    routes.  by_region=False: (sender rank, sender order), the order without header compaction."""
    ks, ids, srcs = [], [], []
    for s, k in enumerate(batches):
        _, _, _, owner, _ = o.route_batch_np(k, spec, full, my_silo=s)
        sel = np.nonzero(np.where(owner == o.M32, s, owner % W) == r)[0]
        if by_region:
            sel = sel[o.region_order(k[sel])]
        ks.append(k[sel]), ids.append(sel), srcs.append(np.full(len(sel), s))
    rk = np.concatenate(ks)
    st, silo, act, _, _ = o.route_batch_np(rk, spec, full, my_silo=r)
    return rk, np.concatenate(ids).astype(np.uint32), np.concatenate(srcs).astype(np.uint32), st, silo, act


@pytest.mark.parametrize("W,by_region", [(2, True), (3, True), (5, True), (3, False)])
def test_route_multi_local_world(gd, W, by_region, monkeypatch):
    """gd_route_multi at W ranks (in-process transport): owner-side arrival order, routes and
    per-activation buckets, and the routes returned to every sender in batch order.  by_region:
    GD_OPT_REGION_PROBE (senders group each chunk by table region, the owner probes region by XCD);
    without it the arrival order is (sender rank, sender order)."""
    monkeypatch.setitem(gd.DEFAULT_OPTIONS, "region_probe", 1 if by_region else 0)
    silos = o.bench_silos(8)
    G = 6000
    reg = o.grain_keys(TC, np.arange(G))
    spec = o.ring_spec(silos, "D")
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    act = np.zeros(G, np.uint32)
    for r in range(W):                     # activation ids local to the owner rank
        act[own % W == r] = np.arange(int((own % W == r).sum()))
    spec, own, es = _local_world(gd, W, "D", silos, reg, act, own)
    rng = np.random.default_rng(W)
    batches = []
    for r in range(W):
        k = o.grain_keys(TC, rng.integers(0, G + 400, size=int(rng.integers(0, 40000)) if r else 33333))
        if len(k) > 50:
            k[::41] = np.array(o.UniqueKey(0, 7, o.type_code_data(o.CAT_SYSTEM_TARGET, 1)).as_tuple(), np.uint64)
        batches.append(k)
    n_act = [int((own % W == r).sum()) for r in range(W)]
    res = _run_ranks([lambda r=r: es[r].route_multi(batches[r], n_act[r], return_routes=True) for r in range(W)])
    full = o.DirectoryArrays(reg, act, own)
    for r in range(W):
        rk, ids, srcs, st, silo, a = _expected_owner_side(batches, spec, full, W, r, by_region=by_region)
        np.testing.assert_array_equal(res[r]["recv_keys"], rk)
        np.testing.assert_array_equal(res[r]["recv_idx"], ids)
        np.testing.assert_array_equal(res[r]["recv_src"], srcs)
        np.testing.assert_array_equal(res[r]["status"], st)
        np.testing.assert_array_equal(res[r]["silo"], silo)
        np.testing.assert_array_equal(res[r]["act"], a)
        wp, wo = o.bucket_stable(a, n_act[r])
        np.testing.assert_array_equal(res[r]["perm"], wp)
        np.testing.assert_array_equal(res[r]["offsets"], wo)
        # routes back at sender r, in batch order = the owner's answer (system targets: r itself)
        st, silo, a, _, _ = o.route_batch_np(batches[r], spec, full, my_silo=r)
        np.testing.assert_array_equal(res[r]["ret_status"], st)
        np.testing.assert_array_equal(res[r]["ret_silo"], silo)
        np.testing.assert_array_equal(res[r]["ret_act"], a)
    for e in es:
        e.comm_destroy()
        e.close()


@pytest.mark.parametrize("by_region", [True, False])
def test_route_multi_local_pipelined_and_forward(gd, by_region, monkeypatch):
    """W = 4: five pipelined device batches per rank (GD_MULTI_KEYS_READY, results checked one
    call later), then the forward hop with activations away from their owners.  Without the region
    order the batches travel with 2-B origin indices (KD_IDX16), which the forward hop carries on."""
    import torch
    monkeypatch.setitem(gd.DEFAULT_OPTIONS, "region_probe", 1 if by_region else 0)
    W, G = 4, 5000
    silos = o.bench_silos(8)
    reg = o.grain_keys(TC, np.arange(G))
    spec = o.ring_spec(silos, "V")
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    act_silo = ((5 * np.arange(G) + 1) % 8).astype(np.uint32)
    host = act_silo % W
    act = np.zeros(G, np.uint32)
    for r in range(W):
        act[host == r] = np.arange(int((host == r).sum()))
    spec, own, es = _local_world(gd, W, "V", silos, reg, act, act_silo)
    full = o.DirectoryArrays(reg, act, act_silo)
    streams = [torch.cuda.Stream() for _ in range(W)]
    for r in range(W):
        es[r].set_stream(streams[r].cuda_stream)
    rng = np.random.default_rng(77)
    batches = [[o.grain_keys(TC, rng.integers(0, G + 300, size=int(rng.integers(1, 30000)))) for _ in range(5)]
               for _ in range(W)]

    def read(rp):
        m = rp.n_recv
        dev = lambda ptr, shape, t: torch.as_tensor(_Cai(ptr, shape, t), device="cuda").cpu().numpy()
        return {"recv_keys": dev(rp.recv_keys, (m, 3), "<i8").view(np.uint64),
                "recv_idx": dev(rp.recv_idx, (m,), "<i4").view(np.uint32),
                "act": dev(rp.act, (m,), "<i4").view(np.uint32), "perm": dev(rp.perm, (m,), "<i4").view(np.uint32),
                "offsets": dev(rp.offsets, (G + 2,), "<i4").view(np.uint32)}

    def pipelined(r):
        dk = [torch.from_numpy(b.view(np.int64).copy()).cuda() for b in batches[r]]
        torch.cuda.synchronize()
        got, prev = [], None
        for i in range(6):
            cur = None
            if i < 5:
                with torch.cuda.stream(streams[r]):
                    cur = es[r].route_multi_device(dk[i].data_ptr(), len(batches[r][i]), G, keys_ready=True)
            if prev is not None:           # batch i-1's result, read after batch i was enqueued
                es[r].synchronize()
                got.append(read(prev))
            prev = cur
        return got

    res = _run_ranks([lambda r=r: pipelined(r) for r in range(W)])
    for i in range(5):
        for r in range(W):
            rk, ids, srcs, st, silo, a = _expected_owner_side([batches[s][i] for s in range(W)], spec, full, W, r,
                                                              by_region=by_region)
            np.testing.assert_array_equal(res[r][i]["recv_keys"], rk, err_msg=f"batch {i} rank {r}")
            np.testing.assert_array_equal(res[r][i]["recv_idx"], ids)
            np.testing.assert_array_equal(res[r][i]["act"], a)
            wp, wo = o.bucket_stable(a, G)
            np.testing.assert_array_equal(res[r][i]["perm"], wp)
            np.testing.assert_array_equal(res[r][i]["offsets"], wo)
    # forward hop: each message ends on its activation's rank (hits) or its owner (the rest)
    n_act = [int((host == r).sum()) for r in range(W)]
    fb = [batches[r][0] for r in range(W)]
    res = _run_ranks([lambda r=r: es[r].route_multi(fb[r], n_act[r], forward=True) for r in range(W)])
    expect = {r: [] for r in range(W)}
    for s in range(W):
        st, silo, a, owner, _ = o.route_batch_np(fb[s], spec, full, my_silo=s)
        orank = np.where(owner == o.M32, s, owner % W)
        final = np.where(st == o.ST_OK, silo % W, orank)
        reg_ = o.table_region_np(fb[s]) if by_region else np.zeros(len(fb[s]), np.uint32)
        for i in range(len(fb[s])):        # (owner rank, sender, region on the owner, sender order)
            expect[int(final[i])].append((int(orank[i]), s, int(reg_[i]), i))
    for r in range(W):
        ex = sorted(expect[r])
        np.testing.assert_array_equal(res[r]["recv_src"], np.array([x[1] for x in ex], np.uint32))
        np.testing.assert_array_equal(res[r]["recv_idx"], np.array([x[3] for x in ex], np.uint32))
        rk = np.array([fb[x[1]][x[3]] for x in ex], np.uint64).reshape(-1, 3)
        np.testing.assert_array_equal(res[r]["recv_keys"], rk)
        st, silo, a, _, _ = o.route_batch_np(rk, spec, full, my_silo=r)
        np.testing.assert_array_equal(res[r]["status"], st)
        np.testing.assert_array_equal(res[r]["act"], a)
        wp, wo = o.bucket_stable(a, n_act[r])
        np.testing.assert_array_equal(res[r]["perm"], wp)
        np.testing.assert_array_equal(res[r]["offsets"], wo)
    for e in es:
        e.comm_destroy()
        e.close()


def test_route_multi_ext_local_world(gd):
    """gd_route_multi_ext at W = 3: KeyExt grains go to the rank owning their KeyExt hash with
    their strings (byte round), host-kept and system-target messages stay with their sender."""
    import keyext as kx
    W, G = 3, 3000
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "R")
    reg = o.grain_keys(TC, np.arange(G))
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    spec, own, es = _local_world(gd, W, "R", silos, reg, np.arange(G, dtype=np.uint32), own)
    stc = o.grain_type_code("UnitTests.GrainInterfaces.IStringKeyGrain")
    tcd = o.type_code_data(o.CAT_KEYEXT_GRAIN, stc)
    names = [(f"user/{i}" + "ü" * (i % 5) + "q" * (i % 40)).encode() for i in range(500)]
    kxd = kx.KeyExtDirectory()
    for i, nm in enumerate(names[:300]):
        owner = int(o.ring_owner_np(spec, np.array([kx.ext_uniform_hash(0, 0, tcd, nm)], np.uint32))[0])
        kxd.add_single_activation((0, 0, tcd), nm, G + i, owner)
        es[owner % W].register_ext(np.array([[0, 0, tcd]], np.uint64), [nm], [G + i], [owner])
    rng = np.random.default_rng(31)
    batches, exts = [], []
    for r in range(W):
        n = 20000 + 777 * r
        k = o.grain_keys(TC, rng.integers(0, G + 200, size=n))
        x = [None] * n
        for i in np.nonzero(rng.random(n) < 0.35)[0]:
            k[i] = (0, 0, tcd)
            x[i] = names[int(rng.integers(0, 500))] if i % 89 else kx.EXT_HOST
        k[5::211] = np.array(o.UniqueKey(0, 7, o.type_code_data(o.CAT_SYSTEM_TARGET, 1)).as_tuple(), np.uint64)
        for i in range(5, n, 211):
            x[i] = None
        batches.append(k)
        exts.append(x)
    bx = [[gd.GD_KEYEXT_HOST if (isinstance(v, str) and v == kx.EXT_HOST) else v for v in x] for x in exts]
    res = _run_ranks([lambda r=r: es[r].route_multi_ext(batches[r], bx[r], G + 300, return_routes=True)
                      for r in range(W)])
    full = o.DirectoryArrays(reg, np.arange(G), own)
    kx_ok = 0
    for r in range(W):
        ks, xs, ids, srcs = [], [], [], []
        for s in range(W):
            _, _, _, owner, _ = kx.route_batch_ext(batches[s], exts[s], spec, full, kxd, my_silo=s)
            sel = np.nonzero(np.where(owner == o.M32, s, owner % W) == r)[0]
            sel = sel[o.region_order(batches[s][sel])]
            ks.append(batches[s][sel]), ids.append(sel), srcs.append(np.full(len(sel), s))
            xs += [exts[s][i] for i in sel]
        rk = np.concatenate(ks)
        np.testing.assert_array_equal(res[r]["recv_keys"], rk)
        np.testing.assert_array_equal(res[r]["recv_idx"], np.concatenate(ids).astype(np.uint32))
        np.testing.assert_array_equal(res[r]["recv_src"], np.concatenate(srcs).astype(np.uint32))
        st, silo, a, _, _ = kx.route_batch_ext(rk, xs, spec, full, kxd, my_silo=r)
        np.testing.assert_array_equal(res[r]["status"], st)
        np.testing.assert_array_equal(res[r]["silo"], silo)
        np.testing.assert_array_equal(res[r]["act"], a)
        wp, wo = o.bucket_stable(a, G + 300)
        np.testing.assert_array_equal(res[r]["perm"], wp)
        np.testing.assert_array_equal(res[r]["offsets"], wo)
        kx_ok += int(((st == o.ST_OK) & (rk[:, 2] == np.uint64(tcd))).sum())
        st, silo, a, _, _ = kx.route_batch_ext(batches[r], exts[r], spec, full, kxd, my_silo=r)
        np.testing.assert_array_equal(res[r]["ret_status"], st)
        np.testing.assert_array_equal(res[r]["ret_act"], a)
    assert kx_ok > 5000            # string-keyed hits were routed on their (remote) owners
    for e in es:
        e.comm_destroy()
        e.close()


@pytest.mark.parametrize("compact,narrow", [("1", "1"), ("1", "0"), ("0", "1")])
def test_route_multi_local_mixed_headers(gd, compact, narrow, monkeypatch):
    """Exchange header compaction: a batch of one grain type with long keys travels as N1s alone
    (k_key_desc / k_recv_expand), 4 B each when every N1 is below 2^32 (GD_OPT_WIRE_HEADERS 2), else 8.
    Ranks here send: one type with small keys (u32 N1s), another type with keys above 2^32 (u64
    N1s, other TCD), guid grains mixed in (full 24-B headers), nothing at all; with compaction off
    (GD_OPT_WIRE_HEADERS 0) everything goes as 24 B.  The results are identical either way."""
    monkeypatch.setitem(gd.DEFAULT_OPTIONS, "wire_headers", 0 if compact == "0" else (2 if narrow == "1" else 1))
    W = 4
    silos = o.bench_silos(8)
    tc2 = o.grain_type_code("UnitTests.Grains.SimpleGrain")
    ka = o.grain_keys(TC, np.arange(3000))
    kb = o.grain_keys(tc2, np.arange(2000) + (1 << 33) + 12345)
    kg = np.array([o.guid_key(f"0d2b3e5a-1111-4c3b-9f4e-aa{i:010d}", o.CAT_GRAIN, TC).as_tuple() for i in range(300)],
                  np.uint64)
    reg = np.concatenate([ka, kb, kg])
    spec = o.ring_spec(silos, "D")
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    act = np.zeros(len(reg), np.uint32)
    for r in range(W):
        act[own % W == r] = np.arange(int((own % W == r).sum()))
    spec, own, es = _local_world(gd, W, "D", silos, reg, act, own)
    rng = np.random.default_rng(8)
    batches = [ka[rng.integers(0, 3000, size=25000)],
               np.concatenate([kb, o.grain_keys(tc2, np.arange(5000, 5100) + (1 << 33))])[rng.integers(0, 2100,
                                                                                                size=17000)],
               reg[rng.integers(0, len(reg), size=21000)],
               np.zeros((0, 3), np.uint64)]
    n_act = [int((own % W == r).sum()) for r in range(W)]
    for e in es:
        e.set_kernel_timing(True)
    res = _run_ranks([lambda r=r: es[r].route_multi(batches[r], n_act[r], return_routes=True) for r in range(W)])
    # every rank receives from the compact ranks 0 and 1 unless compaction is off
    for e in es:
        assert ("k_recv_expand" in e.kernel_times()) == (compact == "1")
    full = o.DirectoryArrays(reg, act, own)
    for r in range(W):
        rk, ids, srcs, st, silo, a = _expected_owner_side(batches, spec, full, W, r, by_region=compact == "1")
        np.testing.assert_array_equal(res[r]["recv_keys"], rk)
        np.testing.assert_array_equal(res[r]["recv_idx"], ids)
        np.testing.assert_array_equal(res[r]["recv_src"], srcs)
        np.testing.assert_array_equal(res[r]["status"], st)
        np.testing.assert_array_equal(res[r]["act"], a)
        wp, wo = o.bucket_stable(a, n_act[r])
        np.testing.assert_array_equal(res[r]["perm"], wp)
        np.testing.assert_array_equal(res[r]["offsets"], wo)
        st, silo, a, _, _ = o.route_batch_np(batches[r], spec, full, my_silo=r)
        np.testing.assert_array_equal(res[r]["ret_status"], st)
        np.testing.assert_array_equal(res[r]["ret_act"], a)
    for e in es:
        e.comm_destroy()
        e.close()


@pytest.mark.parametrize("two_types,big", [(False, False), (True, False), (False, True), (False, "all")])
def test_route_multi_local_no_keys(gd, two_types, big, monkeypatch):
    """GD_MULTI_NO_KEYS at W = 3: with one grain type everywhere the probe reads the compact N1s
    as received (route_n1_device: u32 N1s, or u64 when every sender has a key above 2^32); with two
    types, or u32 and u64 chunks mixed (one sender with big keys), the keys are rebuilt first.
    Results other than recv_keys (left unset) are the same either way."""
    by_region = not big                               # the big-key cases run with 2-B origin indices
    monkeypatch.setitem(gd.DEFAULT_OPTIONS, "region_probe", 1 if by_region else 0)
    W, G = 3, 4000
    silos = o.bench_silos(8)
    tc2 = o.grain_type_code("UnitTests.Grains.SimpleGrain")
    reg = np.concatenate([o.grain_keys(TC, np.arange(G)), o.grain_keys(tc2, np.arange(G)),
                          o.grain_keys(TC, np.arange(G) + (1 << 32))])
    spec = o.ring_spec(silos, "D")
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    act = np.zeros(len(reg), np.uint32)
    for r in range(W):
        act[own % W == r] = np.arange(int((own % W == r).sum()))
    spec, own, es = _local_world(gd, W, "D", silos, reg, act, own)
    rng = np.random.default_rng(12)
    batches = [o.grain_keys(tc2 if (two_types and r == 1) else TC, rng.integers(0, G + 300, size=30000 + r))
               for r in range(W)]
    for r in range(W):
        if big == "all" or (big and r == 1):      # some keys above 2^32: that sender's N1s go as u64
            batches[r][::3, 1] += np.uint64(1 << 32)
    n_act = [int((own % W == r).sum()) for r in range(W)]
    res = _run_ranks([lambda r=r: es[r].route_multi(batches[r], n_act[r], no_keys=True) for r in range(W)])
    full = o.DirectoryArrays(reg, act, own)
    for r in range(W):
        rk, ids, srcs, st, silo, a = _expected_owner_side(batches, spec, full, W, r, by_region=by_region)
        assert res[r]["recv_keys"] is None
        np.testing.assert_array_equal(res[r]["recv_idx"], ids)
        np.testing.assert_array_equal(res[r]["recv_src"], srcs)
        np.testing.assert_array_equal(res[r]["status"], st)
        np.testing.assert_array_equal(res[r]["silo"], silo)
        np.testing.assert_array_equal(res[r]["act"], a)
        wp, wo = o.bucket_stable(a, n_act[r])
        np.testing.assert_array_equal(res[r]["perm"], wp)
        np.testing.assert_array_equal(res[r]["offsets"], wo)
        assert (st == o.ST_OK).sum() > 20000 * 0.9 / W
        with pytest.raises(gd.GrainDispatchError):        # the keys were not kept
            buf = np.empty((len(ids), 3), np.uint64)
            es[r]._c(gd.lib.gd_multi_fetch(es[r].h, gd._ptr(buf), *([None] * 10)))
    for e in es:
        e.comm_destroy()
        e.close()


@pytest.mark.parametrize("idx16", ["1", "0"])
def test_route_multi_local_idx16_mixed(gd, idx16, monkeypatch):
    """2-B origin indices on the wire (KD_IDX16: low 16 bits + per-rank block starts, rebuilt by
    k_recv_idx16) at W = 3 with senders of both widths in one round: rank 1's handle was created
    with GD_OPT_IDX16 0 (4-B indices), ranks 0 and 2 with the parameter; rank 0's batch spans four
    65,536-index blocks with a long one-owner stretch (empty blocks for the other owners), rank 2
    sends nothing.  Owner-side order (sender rank, sender order), routes and buckets against the
    oracle."""
    monkeypatch.setitem(gd.DEFAULT_OPTIONS, "region_probe", 0)
    W, G = 3, 5000
    silos = o.bench_silos(8)
    reg = o.grain_keys(TC, np.arange(G))
    spec = o.ring_spec(silos, "D")
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    act = np.zeros(G, np.uint32)
    for r in range(W):
        act[own % W == r] = np.arange(int((own % W == r).sum()))
    es = []
    for r in range(W):
        e = gd.GrainDispatch(device=0, table_capacity=1 << 13, my_silo=r,
                             options={"idx16": 0 if r == 1 else int(idx16)})
        e.ring_set_silos("D", [(x.ip, x.port, x.gen) for x in silos])
        mine = own % W == r
        e.register(reg[mine], act[mine], own[mine])
        e.set_kernel_timing(True)
        es.append(e)
    gd.GrainDispatch.comm_init_local(es)
    rng = np.random.default_rng(16)
    g0 = rng.integers(0, G + 200, size=230_000)
    by_rank = [np.nonzero(own % W == r)[0] for r in range(W)]
    g0[70_000:150_000] = rng.choice(by_rank[1], size=80_000)      # one owner only: empty blocks elsewhere
    batches = [o.grain_keys(TC, g0), o.grain_keys(TC, rng.integers(0, G, size=40_000)), np.zeros((0, 3), np.uint64)]
    n_act = [int((own % W == r).sum()) for r in range(W)]
    res = _run_ranks([lambda r=r: es[r].route_multi(batches[r], n_act[r]) for r in range(W)])
    for e in es:                       # every rank receives from rank 0
        assert ("k_recv_idx16" in e.kernel_times()) == (idx16 == "1")
    full = o.DirectoryArrays(reg, act, own)
    for r in range(W):
        rk, ids, srcs, st, silo, a = _expected_owner_side(batches, spec, full, W, r, by_region=False)
        np.testing.assert_array_equal(res[r]["recv_keys"], rk)
        np.testing.assert_array_equal(res[r]["recv_idx"], ids)
        np.testing.assert_array_equal(res[r]["recv_src"], srcs)
        np.testing.assert_array_equal(res[r]["status"], st)
        np.testing.assert_array_equal(res[r]["act"], a)
        wp, wo = o.bucket_stable(a, n_act[r])
        np.testing.assert_array_equal(res[r]["perm"], wp)
        np.testing.assert_array_equal(res[r]["offsets"], wo)
    for e in es:
        e.comm_destroy()
        e.close()


def test_route_multi_local_idx16_silent_sender(gd, monkeypatch):
    """a 2-B-index sender with a non-empty batch that sends one owner nothing,
    followed by a higher-ranked 2-B sender whose chunk for that owner spans blocks past 65,536.
    k_recv_idx16 must skip the silent sender's block starts (it sent none) exactly as the host
    layout does, or every later chunk's high 16 bits come from the wrong column.  W = 3, every
    handle with 2-B indices: rank 0 sends only to ranks 0 and 1, rank 1 sends ~100k messages to
    rank 2."""
    monkeypatch.setitem(gd.DEFAULT_OPTIONS, "region_probe", 0)
    monkeypatch.setitem(gd.DEFAULT_OPTIONS, "idx16", 1)
    W, G = 3, 6000
    silos = o.bench_silos(8)
    reg = o.grain_keys(TC, np.arange(G))
    spec = o.ring_spec(silos, "D")
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    act = np.zeros(G, np.uint32)
    for r in range(W):
        act[own % W == r] = np.arange(int((own % W == r).sum()))
    es = []
    for r in range(W):
        e = gd.GrainDispatch(device=0, table_capacity=1 << 14, my_silo=r)
        e.ring_set_silos("D", [(x.ip, x.port, x.gen) for x in silos])
        mine = own % W == r
        e.register(reg[mine], act[mine], own[mine])
        e.set_kernel_timing(True)
        es.append(e)
    gd.GrainDispatch.comm_init_local(es)
    rng = np.random.default_rng(161)
    by_rank = [np.nonzero(own % W == r)[0] for r in range(W)]
    not2 = np.concatenate([by_rank[0], by_rank[1]])
    b0 = rng.choice(not2, size=90_000)                           # n > 0, nothing for owner 2
    b1 = rng.integers(0, G, size=300_000)                        # ~100k for owner 2: blocks 0..4
    b2 = rng.integers(0, G, size=1_000)
    batches = [o.grain_keys(TC, b0), o.grain_keys(TC, b1), o.grain_keys(TC, b2)]
    n_act = [int((own % W == r).sum()) for r in range(W)]
    res = _run_ranks([lambda r=r: es[r].route_multi(batches[r], n_act[r]) for r in range(W)])
    assert "k_recv_idx16" in es[2].kernel_times()
    full = o.DirectoryArrays(reg, act, own)
    for r in range(W):
        rk, ids, srcs, st, silo, a = _expected_owner_side(batches, spec, full, W, r, by_region=False)
        np.testing.assert_array_equal(res[r]["recv_idx"], ids)
        np.testing.assert_array_equal(res[r]["recv_src"], srcs)
        np.testing.assert_array_equal(res[r]["status"], st)
        np.testing.assert_array_equal(res[r]["act"], a)
        wp, wo = o.bucket_stable(a, n_act[r])
        np.testing.assert_array_equal(res[r]["perm"], wp)
        np.testing.assert_array_equal(res[r]["offsets"], wo)
    assert int((res[2]["recv_src"] == 1).sum()) > 65_536
    for e in es:
        e.comm_destroy()
        e.close()
