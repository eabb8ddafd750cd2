"""Batch pipelining (gd_set_bucket_stream): gd_route_bucket_device enqueues each batch's bucketing on a
second stream, so the next batch's route overlaps it.  Several batches routed back to back without a
host synchronisation must give exactly the serial results (the oracle's routes, the stable bucketing),
and a bucketing enqueued on the handle's own stream meanwhile must wait for the bucket stream's scratch.
"""
import numpy as np
import pytest

import oracle as o

pytestmark = pytest.mark.gpu

TC = o.grain_type_code(o.PING_GRAIN_CLASS)


@pytest.fixture(scope="module")
def gd():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    from orleans_amd import graindispatch as g
    return g


def _setup(gd, G):
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    e = gd.GrainDispatch(device=0, table_capacity=2 * G)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    reg = o.grain_keys(TC, np.arange(G))
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    e.register(reg, np.arange(G), owner)
    return e, owner


@pytest.mark.parametrize("G,N", [(1 << 20, 1 << 21), (1 << 14, (1 << 20) + 4099)])
def test_pipelined_batches_match_serial(gd, G, N):
    import torch
    from orleans_amd.sharded import DeviceEngine
    dev = torch.device("cuda:0")
    e, owner = _setup(gd, G)
    eng = DeviceEngine(e, dev, pipeline=True)
    assert eng.bstream is not None and eng.bstream.cuda_stream != eng.stream.cuda_stream
    rng = np.random.default_rng(0x5EED0201)
    batches = []
    # a skewed batch too: one hot activation holds a fifth of the messages
    for b in range(5):
        ks = rng.integers(0, G, size=N)
        if b == 2:
            ks[rng.random(N) < 0.2] = 7
        batches.append(ks)
    with torch.cuda.stream(eng.stream):
        keys = [torch.from_numpy(o.grain_keys(TC, ks).view(np.int64)).to(dev) for ks in batches]
        res = [eng.route_bucket(k, G) for k in keys]          # no host synchronisation between batches
        # a bucketing on the handle's own stream while the bucket stream may still run
        p_main, o_main = eng.bucket(res[-1][2], G)
        eng.stream.wait_stream(eng.bstream)
    torch.cuda.synchronize()
    for ks, (st, silo, act, perm, off) in zip(batches, res):
        assert bool((st == 0).all())
        np.testing.assert_array_equal(act.cpu().numpy().view(np.uint32), ks.astype(np.uint32))
        np.testing.assert_array_equal(silo.cpu().numpy().view(np.uint32), owner[ks])
        wp, wo = o.bucket_stable(ks.astype(np.uint32), G)
        np.testing.assert_array_equal(perm.cpu().numpy().view(np.uint32), wp)
        np.testing.assert_array_equal(off.cpu().numpy().view(np.uint32), wo)
    np.testing.assert_array_equal(p_main.cpu().numpy(), res[-1][3].cpu().numpy())
    np.testing.assert_array_equal(o_main.cpu().numpy(), res[-1][4].cpu().numpy())
    # back to serial: the same results on the handle's stream
    e.set_bucket_stream(None)
    with torch.cuda.stream(eng.stream):
        eng.bstream = None
        st, silo, act, perm, off = eng.route_bucket(keys[0], G)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(perm.cpu().numpy(), res[0][3].cpu().numpy())
    np.testing.assert_array_equal(off.cpu().numpy(), res[0][4].cpu().numpy())
    e.close()


def test_pipelined_batches_with_directory_churn(gd):
    """with the bucketing on the bucket stream, directory batches and other entry
    points enqueued on the handle's stream between pipelined batches must not touch the scratch of a
    bucketing still running (bfence).  Between five pipelined batches: an asynchronous RemoveActivation
    batch, an asynchronous AddSingleActivation batch (gd_dir_unregister_device /
    gd_dir_register_device_async) and a host ring lookup.  Every batch's routes and
    buckets equal the oracle's for the directory as it stood when the batch was routed."""
    import torch
    from orleans_amd.sharded import DeviceEngine
    dev = torch.device("cuda:0")
    G, N, W = 1 << 16, (1 << 20) + 17, 1 << 11
    e, owner = _setup(gd, G)
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    eng = DeviceEngine(e, dev, pipeline=True)
    rng = np.random.default_rng(0x5EED0202)
    reg = o.grain_keys(TC, np.arange(G))
    live = np.ones(G, bool)
    want, res = [], []
    hashes = rng.integers(0, 1 << 32, size=5000, dtype=np.uint64).astype(np.uint32)
    with torch.cuda.stream(eng.stream):
        for b in range(5):
            ks = rng.integers(0, G, size=N)
            keys = torch.from_numpy(o.grain_keys(TC, ks).view(np.int64)).to(dev)
            res.append(eng.route_bucket(keys, G))
            d = o.DirectoryArrays(reg[live], np.arange(G)[live], owner[live])
            w = o.route_batch_np(o.grain_keys(TC, ks), spec, d)
            want.append((w, o.bucket_stable(w[2], G)))
            # churn on the handle's stream while this batch's bucketing may still run
            gone = np.arange(b * W, (b + 1) * W)
            dk = torch.from_numpy(reg[gone].view(np.int64)).to(dev)
            da = torch.from_numpy(gone.astype(np.int32)).to(dev)
            e.unregister_device(dk.data_ptr(), da.data_ptr(), len(gone))
            live[gone] = False
            if b:
                back = np.arange((b - 1) * W, b * W)
                rk = torch.from_numpy(reg[back].view(np.int64)).to(dev)
                rv = torch.from_numpy(np.stack([back, owner[back]], 1).astype(np.int32)).to(dev)
                e.register_device_async(rk.data_ptr(), rv.data_ptr(), len(back))
                live[back] = True
            assert len(e.ring_lookup_hashes(hashes)) == len(hashes)
        eng.stream.wait_stream(eng.bstream)
    torch.cuda.synchronize()
    e.synchronize()                                              # surfaces any deferred device error
    for (w, (wp, wo)), (st, silo, act, perm, off) in zip(want, res):
        np.testing.assert_array_equal(st.cpu().numpy(), w[0])
        np.testing.assert_array_equal(silo.cpu().numpy().view(np.uint32), w[1])
        np.testing.assert_array_equal(act.cpu().numpy().view(np.uint32), w[2])
        np.testing.assert_array_equal(perm.cpu().numpy().view(np.uint32), wp)
        np.testing.assert_array_equal(off.cpu().numpy().view(np.uint32), wo)
    e.close()
