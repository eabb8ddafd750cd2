"""Worker for tests/test_gpu_multi.py: one rank of the in-library RCCL exchange
(gd_comm_init + gd_route_multi), every rank on cuda:0.  Rank 0 writes the RCCL
unique id to <dir>/id; the others wait for it.  Results go to <dir>/rank<r>.npz.
Exit code 77: RCCL refused several ranks on one GPU (the test then skips)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as o                                    # noqa: E402
from orleans_amd import graindispatch as g            # noqa: E402

TC = o.grain_type_code(o.PING_GRAIN_CLASS)
G_TOTAL = 3000


def batch_of(rank, n):
    rng = np.random.default_rng(2000 + rank)
    return o.grain_keys(TC, rng.integers(0, G_TOTAL + 200, size=n))   # ~6% unregistered -> MISS


def main():
    out_dir, world, rank, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    silos = o.bench_silos(8)
    spec = o.ring_spec(silos, "D")
    reg = o.grain_keys(TC, np.arange(G_TOTAL))
    own = o.ring_owner_np(spec, o.jenkins_u64x3_np(reg[:, 2], reg[:, 0], reg[:, 1])).astype(np.uint32)
    mine = np.nonzero(own % world == rank)[0]
    e = g.GrainDispatch(device=0, table_capacity=1 << 13, my_silo=rank)
    e.ring_set_silos("D", [(s.ip, s.port, s.gen) for s in silos])
    e.register(reg[mine], np.arange(len(mine)), own[mine])
    id_path = os.path.join(out_dir, "id")
    if rank == 0:
        uid = g.GrainDispatch.comm_unique_id()
        with open(id_path + ".tmp", "wb") as f:
            f.write(uid)
        os.rename(id_path + ".tmp", id_path)
    else:
        t0 = time.time()
        while not os.path.exists(id_path):
            if time.time() - t0 > 60:
                sys.exit("no unique id from rank 0")
            time.sleep(0.05)
        uid = open(id_path, "rb").read()
    try:
        e.comm_init(uid, world, rank)
    except g.GrainDispatchError as ex:
        print(f"rank {rank}: comm_init failed: {ex}", flush=True)
        sys.exit(77)
    res = e.route_multi(batch_of(rank, n), len(mine), return_routes=True)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
    e.comm_destroy()
    e.close()
    print(f"rank {rank}: ok, received {res['recv_keys'].shape[0]}", flush=True)


if __name__ == "__main__":
    main()
