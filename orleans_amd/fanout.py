"""Follower fan-out cascade (BASELINE cfg 4) on libgraindispatch.

Chirper's publish path (Samples/Chirper/ChirperGrains/ChirperAccount.cs:106-147): a publisher
sends NewChirp to every follower in State.Followers enumeration order (:131-134); each NewChirp
is a grain call that is routed (ring owner + directory probe) and enqueued on the follower's
activation in arrival order.  A cascade repeats that for `hops` rounds: the publishers of
round h+1 are the activations that received a chirp in round h and have not published yet
(BFS frontier), in activation order.

Node u of the follower graph is the grain GrainId(typeCode(ChirperAccount), (long)u); its
activation index in the directory is u (the bench registers it so).

* `FanoutCascade` -- one GPU: per hop one fused expand+route call
  (gd_fanout_route_bucket_device), the activation bucketing, and gd_frontier_next_device.
* `LibraryFanout` -- N GPUs, the whole sharded cascade inside libgraindispatch
  (gd_fanout_multi_device over the library's RCCL communicator): the path a C# host drives; with
  `node_of`, over a partitioned follower graph (gd_fanout_multi_part_device: each rank holds the
  follower lists of the grains it owns, ~1/N of the edges; partition_graph_np / _torch build it).
  (Round 4 removed the torch.distributed form of the same cascade, which duplicated it.)
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import graindispatch as g

CHIRPER_ACCOUNT_CLASS = "Orleans.Samples.Chirper.Grains.ChirperAccount"


@dataclass
class FollowerGraph:
    row_off: torch.Tensor    # (n_nodes+1,) int32 (u32 bit pattern), device
    dst: torch.Tensor        # (E,) int32, device
    n_nodes: int

    @property
    def edges(self) -> int:
        return int(self.dst.shape[0])


def partition_graph_np(row_off: np.ndarray, dst: np.ndarray, nodes: np.ndarray):
    """This rank's part of a follower graph for gd_fanout_multi_part_device: the rows of `nodes`
    (ascending node ids, the grains this rank owns) as a local CSR (row i = local activation i) and
    node_of[i] = nodes[i]."""
    nodes = np.asarray(nodes, dtype=np.int64)
    ro = np.asarray(row_off, dtype=np.int64)
    deg = ro[nodes + 1] - ro[nodes]
    ro_l = np.zeros(nodes.size + 1, np.int64)
    np.cumsum(deg, out=ro_l[1:])
    idx = np.repeat(ro[nodes] - ro_l[:-1], deg) + np.arange(int(ro_l[-1]), dtype=np.int64)
    return ro_l.astype(np.uint32), np.asarray(dst, dtype=np.uint32)[idx], nodes.astype(np.uint32)


def partition_graph_torch(row_off: torch.Tensor, dst: torch.Tensor, nodes: torch.Tensor):
    """partition_graph_np on the device (int64 row offsets, int32 node ids): (row_off_local int32 bit
    pattern, dst_local int32, node_of int32)."""
    nodes = nodes.long()
    ro = row_off.long()
    deg = ro[nodes + 1] - ro[nodes]
    ro_l = torch.zeros(nodes.numel() + 1, dtype=torch.int64, device=nodes.device)
    torch.cumsum(deg, 0, out=ro_l[1:])
    total = int(ro_l[-1].item())
    idx = torch.repeat_interleave(ro[nodes] - ro_l[:-1], deg, output_size=total)
    idx += torch.arange(total, dtype=torch.int64, device=nodes.device)
    return ro_l.to(torch.int32), dst[idx].contiguous(), nodes.to(torch.int32)


def upload_graph(row_off: np.ndarray, dst: np.ndarray, device) -> FollowerGraph:
    ro = torch.from_numpy(np.ascontiguousarray(row_off, dtype=np.uint32).view(np.int32)).to(device)
    d = np.ascontiguousarray(dst, dtype=np.uint32)
    if d.size == 0:
        d = np.zeros(1, dtype=np.uint32)      # keep a valid pointer; row_off says 0 edges
    return FollowerGraph(ro, torch.from_numpy(d.view(np.int32)).to(device), len(row_off) - 1)


@dataclass
class HopResult:
    frontier: torch.Tensor     # publishers of this hop (this rank's share when sharded)
    target: Optional[torch.Tensor]   # (M,) follower node per message (arrival order)
    sender: torch.Tensor       # (M,) publisher node per message
    src_rank: Optional[torch.Tensor]  # (M,) sending rank (sharded only)
    status: torch.Tensor       # (M,) uint8
    silo: torch.Tensor         # (M,) int32
    act: torch.Tensor          # (M,) int32
    perm: torch.Tensor         # (M,) int32: stable per-activation order
    offsets: torch.Tensor      # (n_act+2,) int32

    @property
    def messages(self) -> int:
        return int(self.sender.shape[0])


class DeviceFanoutEngine:
    """libgraindispatch fan-out entry points on torch-allocated HBM, on a dedicated stream."""

    def __init__(self, dispatch: g.GrainDispatch, device: torch.device, type_code: int,
                 stream: Optional[torch.cuda.Stream] = None, keep_target: bool = True):
        self.gd = dispatch
        self.device = device
        self.type_code = type_code
        self.keep_target = keep_target
        self.stream = stream or torch.cuda.Stream(device)
        self.gd.set_stream(self.stream.cuda_stream)

    def _empty(self, n, dtype=torch.int32):
        return torch.empty(n, dtype=dtype, device=self.device)

    def count(self, graph: FollowerGraph, frontier: torch.Tensor) -> int:
        nf = int(frontier.shape[0])
        return self.gd.fanout_expand_device(graph.row_off.data_ptr(), graph.dst.data_ptr(), graph.n_nodes,
                                            frontier.data_ptr() if nf else 0, nf, None, None, 0)

    def expand(self, graph: FollowerGraph, frontier: torch.Tensor):
        nf = int(frontier.shape[0])
        m = self.count(graph, frontier)
        target, sender = self._empty(m), self._empty(m)
        if m:
            got = self.gd.fanout_expand_device(graph.row_off.data_ptr(), graph.dst.data_ptr(), graph.n_nodes,
                                               frontier.data_ptr(), nf, target.data_ptr(), sender.data_ptr(), m)
            assert got == m
        return target, sender

    def expand_route_bucket(self, graph: FollowerGraph, frontier: torch.Tensor, n_act: int,
                            capacity: Optional[int] = None):
        """Fused hop on one GPU.  capacity: known upper bound on the hop's messages (skips the
        size query); None = ask the library first."""
        nf = int(frontier.shape[0])
        m = self.count(graph, frontier) if capacity is None else capacity
        target = self._empty(m) if self.keep_target else None
        sender, silo, act, perm = self._empty(m), self._empty(m), self._empty(m), self._empty(m)
        st = self._empty(m, torch.uint8)
        off = self._empty(n_act + 2)
        got = self.gd.fanout_route_bucket_device(
            graph.row_off.data_ptr(), graph.dst.data_ptr(), graph.n_nodes, frontier.data_ptr() if nf else 0, nf,
            self.type_code, n_act, target.data_ptr() if target is not None else None, sender.data_ptr(),
            silo.data_ptr(), act.data_ptr(), st.data_ptr(), perm.data_ptr(), off.data_ptr(), m)
        if got != m:
            sl = slice(0, got)
            target = target[sl] if target is not None else None
            sender, silo, act, perm, st = sender[sl], silo[sl], act[sl], perm[sl], st[sl]
        return target, sender, st, silo, act, perm, off

    def pack_nodes_by_shard(self, nodes: torch.Tensor, payload: torch.Tensor, n_shards: int):
        n = int(nodes.shape[0])
        sn, sp, counts = self._empty(n), self._empty(n), self._empty(n_shards)
        self.gd.pack_nodes_by_shard_device(nodes.data_ptr(), payload.data_ptr(), n, self.type_code, n_shards,
                                           sn.data_ptr(), sp.data_ptr(), counts.data_ptr())
        return sn, sp, counts

    def route_nodes_bucket(self, nodes: torch.Tensor, n_act: int):
        n = int(nodes.shape[0])
        silo, act, perm = self._empty(n), self._empty(n), self._empty(n)
        st = self._empty(n, torch.uint8)
        off = self._empty(n_act + 2)
        if n:
            self.gd.route_nodes_device(nodes.data_ptr(), n, self.type_code, silo.data_ptr(), act.data_ptr(),
                                       st.data_ptr())
        self.gd.bucket_device(act.data_ptr(), n, n_act, perm.data_ptr(), off.data_ptr())
        return st, silo, act, perm, off

    def new_visited(self, n_act: int) -> torch.Tensor:
        return torch.zeros(n_act, dtype=torch.uint8, device=self.device)

    def mark_visited(self, visited: torch.Tensor, nodes: torch.Tensor):
        ok = nodes[(nodes >= 0) & (nodes < visited.shape[0])].long()
        visited[ok] = 1

    def frontier_next(self, offsets: torch.Tensor, n_act: int, visited: torch.Tensor) -> torch.Tensor:
        out = self._empty(max(n_act, 1))
        k = self.gd.frontier_next_device(offsets.data_ptr(), n_act, visited.data_ptr(), out.data_ptr())
        return out[:k]

    def context(self):
        """Torch work of a cascade runs on the library's stream (allocations included)."""
        return torch.cuda.stream(self.stream)

    def synchronize(self):
        self.stream.synchronize()


class FanoutCascade:
    """All hops on one GPU (world size 1)."""

    def __init__(self, engine: DeviceFanoutEngine, graph: FollowerGraph, n_act: int):
        self.engine, self.graph, self.n_act = engine, graph, n_act

    def run(self, seeds: torch.Tensor, hops: int) -> List[HopResult]:
        with self.engine.context():
            return self._run(seeds, hops)

    def _run(self, seeds: torch.Tensor, hops: int) -> List[HopResult]:
        eng = self.engine
        visited = eng.new_visited(self.n_act)
        frontier = seeds.to(device=eng.device, dtype=torch.int32)
        eng.mark_visited(visited, frontier)
        out = []
        for h in range(hops):
            # from hop 1 on the frontier holds distinct publishers: at most `edges` messages
            cap = self.graph.edges if h > 0 else None
            target, sender, st, silo, act, perm, off = eng.expand_route_bucket(self.graph, frontier, self.n_act, cap)
            out.append(HopResult(frontier, target, sender, None, st, silo, act, perm, off))
            frontier = eng.frontier_next(off, self.n_act, visited)
        return out


class LibraryCascade:
    """All hops on one GPU inside libgraindispatch (gd_fanout_cascade_device): one host read-back a hop
    instead of the two of FanoutCascade's per-hop calls.  Node u = activation u."""

    def __init__(self, engine: DeviceFanoutEngine, graph: FollowerGraph, n_act: int):
        self.engine, self.graph, self.n_act = engine, graph, n_act

    def run(self, seeds: torch.Tensor, hops: int) -> List["LibraryHop"]:
        ns = int(seeds.shape[0])
        with self.engine.context():
            raw = self.engine.gd.fanout_cascade_device(self.graph.row_off.data_ptr(), self.graph.dst.data_ptr(),
                                                       self.graph.n_nodes, seeds.data_ptr() if ns else 0, ns,
                                                       self.engine.type_code, self.n_act, hops)
        return [LibraryHop(r) for r in raw]

    def fetch(self, hops: List["LibraryHop"]) -> List[dict]:
        return [self.engine.gd.fanout_multi_fetch(i, h.raw, self.n_act) for i, h in enumerate(hops)]


class LibraryHop:
    """One hop of gd_fanout_multi_device on this rank: counts, plus the library's device pointers
    (valid until the next cascade on the handle)."""

    def __init__(self, raw: "g.gd_fanout_hop"):
        self.raw = raw
        self.n_frontier = int(raw.n_frontier)
        self.n_recv = int(raw.n_recv)
        self.n_sent = int(raw.n_sent)

    @property
    def messages(self) -> int:
        return self.n_recv


class LibraryFanout:
    """The sharded cascade inside libgraindispatch (gd_comm_init + gd_fanout_multi_device): expand,
    partition by owner rank, one grouped RCCL send/recv round per hop, route + bucket on the owner,
    next frontier -- all in the library on the engine's stream.  torch.distributed only hands the
    RCCL unique id to the other ranks."""

    def __init__(self, engine: DeviceFanoutEngine, graph: FollowerGraph, n_act: int,
                 group: Optional[dist.ProcessGroup] = None, node_of: Optional[torch.Tensor] = None):
        """node_of: `graph` is this rank's partition (partition_graph_*: row i = local activation i,
        node node_of[i], n_act = its rows) -- gd_fanout_multi_part_device; None: the replicated graph."""
        self.engine, self.graph, self.n_act, self.node_of = engine, graph, n_act, node_of
        world, rank = dist.get_world_size(group), dist.get_rank(group)
        uid = torch.zeros(g.GD_COMM_ID_BYTES, dtype=torch.uint8)
        if rank == 0:
            uid = torch.frombuffer(bytearray(g.GrainDispatch.comm_unique_id()), dtype=torch.uint8)
        t = uid.to(engine.device) if dist.get_backend(group) == "nccl" else uid
        dist.broadcast(t, src=0, group=group)
        engine.gd.comm_init(bytes(t.cpu().numpy().tobytes()), world, rank)

    def run(self, seeds: torch.Tensor, hops: int) -> List[LibraryHop]:
        ns = int(seeds.shape[0])
        with self.engine.context():
            if self.node_of is not None:
                raw = self.engine.gd.fanout_multi_part_device(
                    self.graph.row_off.data_ptr(), self.graph.dst.data_ptr(), self.graph.n_nodes,
                    self.node_of.data_ptr(), seeds.data_ptr() if ns else 0, ns, self.engine.type_code, hops)
            else:
                raw = self.engine.gd.fanout_multi_device(self.graph.row_off.data_ptr(), self.graph.dst.data_ptr(),
                                                         self.graph.n_nodes, seeds.data_ptr() if ns else 0, ns,
                                                         self.engine.type_code, self.n_act, hops)
        return [LibraryHop(r) for r in raw]

    def fetch(self, hops: List[LibraryHop]) -> List[dict]:
        """Host copies of every hop of the last cascade (gd_fanout_multi_fetch)."""
        return [self.engine.gd.fanout_multi_fetch(i, h.raw, self.n_act) for i, h in enumerate(hops)]

    def close(self):
        self.engine.gd.comm_destroy()
