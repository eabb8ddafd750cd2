"""Wall time of cfg 2's directory batches (1 % RemoveActivation + 1 % AddSingleActivation, enqueued)
against the launch floor of tiny kernels on this stack.  profiles/r06_dir_batch_probe.json holds a run
(with a since-removed switch that skipped the three gated claim passes: both_nogate)."""
import json, os, sys, time
import numpy as np, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from orleans_amd import graindispatch as g
from orleans_amd.workloads import grain_keys_torch
SILOS = [(f"10.0.0.{i + 1}", 11111, gen) for i, gen in enumerate([138558, 165678, 215136, 61804, 17808, 48728, 207265, 76820])]
G = 1 << 20
dev = torch.device("cuda:0")
tc = g.calculate_id_hash("BenchmarkGrains.Ping.PingGrain")
tcd = (3 << 56) + ((tc & 0xFFFFFFFFFFFFFFFF) & 0x00FFFFFFFFFFFFFF)
e = g.GrainDispatch(device=0, table_capacity=2 * G, my_silo=0, kernel_timing=False)
e.ring_set_silos("D", SILOS)
allk = grain_keys_torch(tcd, torch.arange(G, device=dev), dev)
own = torch.empty(G, dtype=torch.int32, device=dev)
e.ring_owner_device(allk.data_ptr(), G, own.data_ptr())
vals = torch.stack([torch.arange(G, device=dev, dtype=torch.int32), own], 1).contiguous()
e.register_device(allk.data_ptr(), vals.data_ptr(), G)
B = G // 100
perm = torch.from_numpy(np.random.default_rng(7).permutation(G).astype(np.int64)).to(dev)
K = [allk[perm[i * B:(i + 1) * B]].contiguous() for i in range(40)]
A = [perm[i * B:(i + 1) * B].to(torch.int32).contiguous() for i in range(40)]
V = [vals[perm[i * B:(i + 1) * B]].contiguous() for i in range(40)]
torch.cuda.synchronize()
res = {}
def run(name, fn, steps=40):
    for s in range(5): fn(s)
    torch.cuda.synchronize(); t0 = time.perf_counter()
    for s in range(5, 5 + steps): fn(s)
    torch.cuda.synchronize()
    res[name] = round((time.perf_counter() - t0) / steps * 1e3, 4)
def unreg(s):
    i = s % 39; e.unregister_device(K[i].data_ptr(), A[i].data_ptr(), B)
def both(s):
    i = s % 39; e.unregister_device(K[i].data_ptr(), A[i].data_ptr(), B); e.register_device_async(K[i].data_ptr(), V[i].data_ptr(), B)
def empty(s):
    e.unregister_device(K[0].data_ptr(), A[0].data_ptr(), 0)
run("both", both)
run("unreg_only_then_rereg", lambda s: (unreg(s), e.register_device_async(K[s % 39].data_ptr(), V[s % 39].data_ptr(), B)))
# per-launch floor: a trivial device op
x = torch.zeros(1, device=dev)
run("8_tiny_torch_kernels", lambda s: [x.add_(1) for _ in range(8)])
run("1_tiny_torch_kernel", lambda s: x.add_(1))
e.synchronize()
print(json.dumps(res), flush=True)
e.close()
