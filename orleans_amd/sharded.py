"""Directory sharded by ring owner across GPUs (one process per GPU).

The mirror of Orleans' per-silo directory partitions (GrainDirectoryPartition,
LocalGrainDirectory.cs:477-545) and of its per-target-silo outbound queues
(OutboundMessageQueue.cs:54-131): every rank owns the directory entries of the
silos it hosts (silo s lives on rank s % world); a batch of message headers is
partitioned by owner rank (stable), exchanged with one all-to-all-v, then
routed (directory probe) and bucketed per activation on the owner.

Exchange = torch.distributed all_to_all_single: RCCL over xGMI on MI355X
(backend "nccl"), gloo in the CPU tests.  This is the cross-check of the library's own exchange
(LibraryRouter: gd_route_multi_device, the product path); membership handoffs are the library's
gd_dir_handoff_multi only (GrainInfo.Merge semantics, GrainDirectoryPartition.cs:139-179).
The local steps run through an
engine object; `DeviceEngine` is the product engine (libgraindispatch device
entry points on torch-allocated HBM buffers).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from . import graindispatch as g


@dataclass
class ShardedResult:
    recv_keys: Optional[torch.Tensor]  # (M,3) int64 -- headers this rank owns, arrival order (None: no_keys)
    recv_idx: Optional[torch.Tensor]   # (M,) int32 -- index in the sender's batch (None: world 1, identity)
    recv_src: Optional[torch.Tensor]   # (M,) int32 -- sender rank (None: world 1, all rank 0)
    status: torch.Tensor        # (M,) uint8
    silo: torch.Tensor          # (M,) int32 (uint32 bit pattern)
    act: torch.Tensor           # (M,) int32 (uint32 bit pattern)
    perm: torch.Tensor          # (M,) int32: stable per-activation order of recv positions
    offsets: torch.Tensor       # (n_act+2,) int32


class DeviceEngine:
    """libgraindispatch on this rank's GPU, driven through the *_device C-ABI
    entry points on the current torch stream."""

    def __init__(self, dispatch: g.GrainDispatch, device: torch.device, stream: Optional[torch.cuda.Stream] = None,
                 pipeline: bool = False):
        self.gd = dispatch
        self.device = device
        # A dedicated (non-null) stream: torch's legacy default stream has handle 0,
        # which the C ABI reads as "use the library's own stream".  Callers run
        # their torch work under `with torch.cuda.stream(engine.stream)`.
        self.stream = stream or torch.cuda.Stream(device)
        self.gd.set_stream(self.stream.cuda_stream)
        # pipeline: route_bucket's bucketing on a second stream (gd_set_bucket_stream), so batch i + 1's
        # route overlaps batch i's bucketing; its outputs are recorded on that stream for the allocator
        self.bstream = torch.cuda.Stream(device) if pipeline else None
        if self.bstream is not None:
            self.gd.set_bucket_stream(self.bstream.cuda_stream)

    def pack_by_shard(self, keys: torch.Tensor, n_shards: int):
        n = keys.shape[0]
        send_keys = torch.empty_like(keys)
        send_idx = torch.empty(n, dtype=torch.int32, device=self.device)
        counts = torch.empty(n_shards, dtype=torch.int32, device=self.device)
        self.gd.pack_by_shard_device(keys.data_ptr(), n, n_shards, send_keys.data_ptr(), send_idx.data_ptr(),
                                     counts.data_ptr())
        return send_keys, send_idx, counts

    def route(self, keys: torch.Tensor):
        n = keys.shape[0]
        dev = self.device
        st = torch.empty(n, dtype=torch.uint8, device=dev)
        silo = torch.empty(n, dtype=torch.int32, device=dev)
        act = torch.empty(n, dtype=torch.int32, device=dev)
        self.gd.route_device(keys.data_ptr(), n, silo.data_ptr(), act.data_ptr(), st.data_ptr())
        return st, silo, act

    def bucket(self, act: torch.Tensor, n_act: int):
        n = act.shape[0]
        perm = torch.empty(n, dtype=torch.int32, device=self.device)
        off = torch.empty(n_act + 2, dtype=torch.int32, device=self.device)
        self.gd.bucket_device(act.data_ptr(), n, n_act, perm.data_ptr(), off.data_ptr())
        return perm, off

    def pack_routes_by_rank(self, keys: torch.Tensor, st: torch.Tensor, silo: torch.Tensor, n_shards: int,
                            my_rank: int):
        n = keys.shape[0]
        send_keys = torch.empty_like(keys)
        send_pos = torch.empty(n, dtype=torch.int32, device=self.device)
        counts = torch.empty(n_shards, dtype=torch.int32, device=self.device)
        self.gd.pack_routes_by_rank_device(keys.data_ptr(), st.data_ptr(), silo.data_ptr(), n, n_shards, my_rank,
                                           send_keys.data_ptr(), send_pos.data_ptr(), counts.data_ptr())
        return send_keys, send_pos, counts

    def route_bucket(self, keys: torch.Tensor, n_act: int):
        """Route + bucket on the engine's stream.  Pipeline mode: the bucketing runs on `bstream` after the
        route, and perm / offsets (and act's last reader) are done only once `bucket_done_event()` is --
        a caller reading them on another stream waits on that event (or on bstream) first."""
        n = keys.shape[0]
        dev = self.device
        st = torch.empty(n, dtype=torch.uint8, device=dev)
        silo = torch.empty(n, dtype=torch.int32, device=dev)
        act = torch.empty(n, dtype=torch.int32, device=dev)
        perm = torch.empty(n, dtype=torch.int32, device=dev)
        off = torch.empty(n_act + 2, dtype=torch.int32, device=dev)
        self.gd.route_bucket_device(keys.data_ptr(), n, n_act, silo.data_ptr(), act.data_ptr(), st.data_ptr(),
                                    perm.data_ptr(), off.data_ptr())
        if self.bstream is not None:
            for t in (act, perm, off):
                t.record_stream(self.bstream)
        return st, silo, act, perm, off

    def bucket_done_event(self):
        """An event the caller's stream can wait on for the last route_bucket's buckets (pipeline mode)."""
        ev = torch.cuda.Event()
        ev.record(self.bstream if self.bstream is not None else self.stream)
        return ev


class ShardedRouter:
    """`stage_via_cpu` is a rehearsal mode only (several ranks sharing one GPU with
    the gloo backend): the all-to-all then runs on host copies of the buffers."""

    def __init__(self, engine, group: Optional[dist.ProcessGroup] = None, stage_via_cpu: bool = False):
        self.engine = engine
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.stage_via_cpu = stage_via_cpu

    def _a2a(self, out: torch.Tensor, inp: torch.Tensor, out_splits=None, in_splits=None):
        if self.stage_via_cpu and out.device.type != "cpu":
            o_cpu = torch.empty(out.shape, dtype=out.dtype)
            dist.all_to_all_single(o_cpu, inp.cpu(), out_splits, in_splits, group=self.group)
            out.copy_(o_cpu)
        else:
            dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def exchange(self, keys: torch.Tensor):
        """Stable partition by owner rank + all-to-all-v of the headers."""
        send_keys, send_idx, counts = self.engine.pack_by_shard(keys, self.world)
        counts64 = counts.to(torch.int64)
        recv_counts = torch.empty_like(counts64)
        self._a2a(recv_counts, counts64)
        in_splits = counts64.tolist()
        out_splits = recv_counts.tolist()
        m = int(sum(out_splits))
        recv_keys = torch.empty((m, 3), dtype=keys.dtype, device=keys.device)
        self._a2a(recv_keys, send_keys, out_splits, in_splits)
        recv_idx = torch.empty(m, dtype=torch.int32, device=keys.device)
        self._a2a(recv_idx, send_idx, out_splits, in_splits)
        recv_src = torch.repeat_interleave(torch.arange(self.world, dtype=torch.int32, device=keys.device),
                                           recv_counts.to(keys.device))
        return recv_keys, recv_idx, recv_src

    def _a2a_v(self, tensors, in_splits, out_splits):
        outs = []
        for t in tensors:
            o = torch.empty((int(sum(out_splits)),) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
            self._a2a(o, t, out_splits, in_splits)
            outs.append(o)
        return outs

    def route_bucket(self, keys: torch.Tensor, n_act: int, forward: bool = False) -> ShardedResult:
        """forward=False: the benchmark's co-location (activation silo = directory owner): probe and
        bucket on the owner.  forward=True: the general case -- probe on the owner, then directory
        hits travel on to the rank hosting their activation (silo % world; the send to
        ActivationAddress.Silo after a remote lookup, LocalGrainDirectory.cs:920,
        OutboundMessageQueue.cs:125) and are bucketed there; other statuses stay on the owner.
        One grain has one owner, so each activation still sees (sender rank, sender order).  With the
        engine in pipeline mode the returned perm / offsets are complete only once
        `engine.bucket_done_event()` is: a reader on another stream waits on it first."""
        if self.world == 1:
            # no exchange: arrival order is the batch order, all from this rank
            recv_keys, recv_idx, recv_src = keys, None, None
        else:
            recv_keys, recv_idx, recv_src = self.exchange(keys)
        if not forward or self.world == 1:
            st, silo, act, perm, off = self.engine.route_bucket(recv_keys, n_act)
            return ShardedResult(recv_keys, recv_idx, recv_src, st, silo, act, perm, off)
        st, silo, act = self.engine.route(recv_keys)
        send_keys, send_pos, counts = self.engine.pack_routes_by_rank(recv_keys, st, silo, self.world, self.rank)
        pos = send_pos.long()
        counts64 = counts.to(torch.int64)
        recv_counts = torch.empty_like(counts64)
        self._a2a(recv_counts, counts64)
        in_splits, out_splits = counts64.tolist(), recv_counts.tolist()
        keys2, idx2, src2, silo2, act2, st2 = self._a2a_v(
            [send_keys, recv_idx[pos], recv_src[pos], silo[pos], act[pos], st[pos]], in_splits, out_splits)
        perm, off = self.engine.bucket(act2, n_act)
        return ShardedResult(keys2, idx2, src2, st2, silo2, act2, perm, off)


class _DevView:
    """A torch view of library-owned HBM (__cuda_array_interface__, no copy)."""

    def __init__(self, ptr: int, shape, typestr: str):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr, "data": (int(ptr), False),
                                         "version": 3, "strides": None}


def _view(ptr: int, shape, typestr: str, device) -> torch.Tensor:
    if not ptr or 0 in tuple(shape):
        dt = {"<i4": torch.int32, "<i8": torch.int64, "|u1": torch.uint8}[typestr]
        return torch.empty(shape, dtype=dt, device=device)
    return torch.as_tensor(_DevView(ptr, shape, typestr), device=device)


class LibraryRouter:
    """The exchange inside libgraindispatch (gd_comm_init + gd_route_multi_device): the
    partition, the grouped RCCL send/recv of headers and origin indices, the probe and the
    bucketing all run in the library on the engine's stream -- the path a C# host drives
    through P/Invoke.  torch.distributed only hands the RCCL unique id to the other ranks."""

    def __init__(self, engine: DeviceEngine, group: Optional[dist.ProcessGroup] = None):
        self.engine = engine
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        dev = engine.device
        uid = torch.zeros(g.GD_COMM_ID_BYTES, dtype=torch.uint8)
        if self.rank == 0:
            uid = torch.frombuffer(bytearray(g.GrainDispatch.comm_unique_id()), dtype=torch.uint8)
        # the backend may need the id on the device (nccl) or the host (gloo)
        on_dev = dist.get_backend(group) == "nccl"
        t = uid.to(dev) if on_dev else uid
        dist.broadcast(t, src=0, group=group)
        engine.gd.comm_init(bytes(t.cpu().numpy().tobytes()), self.world, self.rank)
        self.keys_ready = False
        self.no_keys = False        # GD_MULTI_NO_KEYS: recv_keys None, messages known by (src, idx)

    def route_bucket(self, keys: torch.Tensor, n_act: int, return_routes: bool = False,
                     keys_ready: Optional[bool] = None) -> ShardedResult:
        """keys_ready: `keys` are complete already (their producer was synchronised), so this
        batch's partition + exchange may overlap the previous batch's probe + bucketing.  The
        returned views stay valid through the next call.  None: the router's `keys_ready`."""
        n = keys.shape[0]
        keys_ready = self.keys_ready if keys_ready is None else keys_ready
        r = self.engine.gd.route_multi_device(keys.data_ptr(), n, n_act, return_routes, keys_ready,
                                              no_keys=self.no_keys)
        m, dev = r.n_recv, self.engine.device
        rk = _view(r.recv_keys, (m, 3), "<i8", dev) if r.recv_keys or m == 0 else None
        return ShardedResult(rk, _view(r.recv_idx, (m,), "<i4", dev),
                             _view(r.recv_src, (m,), "<i4", dev), _view(r.status, (m,), "|u1", dev),
                             _view(r.silo, (m,), "<i4", dev), _view(r.act, (m,), "<i4", dev),
                             _view(r.perm, (m,), "<i4", dev), _view(r.offsets, (n_act + 2,), "<i4", dev))

    def close(self):
        self.engine.gd.comm_destroy()


def _canonical(r: ShardedResult):
    """The owner-side result keyed by message identity (sender rank, index in the sender's batch),
    free of the arrival order: the messages sorted by identity with their keys and routes, and each
    activation's queue as the identities of its messages in bucket order."""
    m = r.status.shape[0]
    dev = r.status.device
    idx = r.recv_idx.long() if r.recv_idx is not None else torch.arange(m, device=dev)
    src = r.recv_src.long() if r.recv_src is not None else torch.zeros(m, dtype=torch.long, device=dev)
    ident = src * (1 << 32) + idx
    order = torch.argsort(ident)
    q = ident[r.perm.long()]
    # the trailing bucket (unrouted messages, many grains) holds them in arrival order: compare as a set
    u = int(r.offsets[-2]) if r.offsets.numel() >= 2 else m
    q = torch.cat([q[:u], torch.sort(q[u:]).values])
    out = [ident[order], r.status[order], r.silo[order], r.act[order], q, r.offsets]
    if r.recv_keys is not None:
        out.append(r.recv_keys[order])
    return out


def same_result(a: ShardedResult, b: ShardedResult) -> bool:
    """The same owner-side results for the same batch (both routers): every message with the same
    key and route, every activation's queue with the same messages in the same order, the same
    offsets.  The two routers' arrival orders may differ (gd_route_multi groups a sender's chunk
    by table region; the per-activation order (sender rank, sender order) is the same)."""
    if a.status.shape != b.status.shape:
        return False
    ca, cb = _canonical(a), _canonical(b)
    return len(ca) == len(cb) and all(torch.equal(x, y) for x, y in zip(ca, cb))


def silo_rank(silo: int, world: int) -> int:
    """Which rank hosts (owns the directory partition of) a silo."""
    return silo % world
