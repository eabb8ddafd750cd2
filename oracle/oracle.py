"""CPU oracle for the Orleans grain-dispatch hot path -- TEST INFRASTRUCTURE ONLY.

This module is a restatement, in Python/numpy, of the C# algorithms on the
Orleans message-dispatch path (ring lookup, directory probe, per-activation
bucketing).  It is the *checker*: only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it.  The product path
(``orleans_amd`` + ``libgraindispatch.so``) never routes through it.

Parity status.  The reference (rikbosch/orleans, Orleans 2.0, pure C#) cannot
be compiled or run in this image (no dotnet/mono/csc), and its own tests hold
no numeric known-answer vectors for these hashes.  The oracle is therefore
pinned by (1) the reference's structural tests, restated in
``tests/test_oracle.py``:
  * ``ID_HashCorrectness``  test/NonSilo.Tests/General/Identifiertests.cs:278-293
  * ``SiloAddressGetUniformHashCodes``  Identifiertests.cs:51-68
  * ``UniqueKeyToByteArray``  Identifiertests.cs:32-48
  * ``RingStandalone_*`` range tiling  test/NonSilo.Tests/General/RingTests_Standalone.cs:15-70,171-261
(2) FIPS 180-4 test vectors for the SHA-256 that the silo / type-code hashes
use, and (3) a second, independent C restatement (``oracle/cpu_ref.c``)
that must agree bit-for-bit.  Absolute hash values are "pinned by source
text + structure", not by a reference run.

Every function cites the reference file:line it restates (paths relative to
the reference root).
"""
from __future__ import annotations

import hashlib
import ipaddress
import struct
import uuid
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

M32 = 0xFFFFFFFF
M64 = 0xFFFFFFFFFFFFFFFF

# UniqueKey.Category  src/Orleans.Core.Abstractions/IDs/UniqueKey.cs:17-26
CAT_NONE, CAT_SYSTEM_TARGET, CAT_SYSTEM_GRAIN, CAT_GRAIN, CAT_CLIENT = 0, 1, 2, 3, 4
CAT_KEYEXT_GRAIN, CAT_GEO_CLIENT = 6, 7

# Per-message routing status (the boundary's out_status codes, include/graindispatch.h)
ST_OK, ST_MISS, ST_SYSTEM_TARGET, ST_MEMBERSHIP, ST_KEYEXT = 0, 1, 2, 3, 4
ST_MULTI_ACT = 7               # several activations: the C# random selection (RandomPlacementDirector.cs:33-53)
ACT_MULTI = 0xFFFFFFFE         # directory value of a multi-activation grain (gd_dir_upsert)

# ---------------------------------------------------------------------------
# L0: Jenkins hash   src/Orleans.Core.Abstractions/IDs/JenkinsHash.cs
# ---------------------------------------------------------------------------


def _mix(a: int, b: int, c: int) -> Tuple[int, int, int]:
    """JenkinsHash.Mix, JenkinsHash.cs:11-22 (uint32 wraparound)."""
    a = (a - b - c) & M32; a ^= c >> 13
    b = (b - c - a) & M32; b ^= (a << 8) & M32
    c = (c - a - b) & M32; c ^= b >> 13
    a = (a - b - c) & M32; a ^= c >> 12
    b = (b - c - a) & M32; b ^= (a << 16) & M32
    c = (c - a - b) & M32; c ^= b >> 5
    a = (a - b - c) & M32; a ^= c >> 3
    b = (b - c - a) & M32; b ^= (a << 10) & M32
    c = (c - a - b) & M32; c ^= b >> 15
    return a, b, c


def jenkins_bytes(data: bytes) -> int:
    """JenkinsHash.ComputeHash(byte[]), JenkinsHash.cs:25-74."""
    n = len(data)
    a = b = 0x9E3779B9
    c = 0
    i = 0
    while i + 12 <= n:
        a = (a + int.from_bytes(data[i:i + 4], "little")) & M32
        b = (b + int.from_bytes(data[i + 4:i + 8], "little")) & M32
        c = (c + int.from_bytes(data[i + 8:i + 12], "little")) & M32
        a, b, c = _mix(a, b, c)
        i += 12
    c = (c + n) & M32
    # tail: a gets bytes 0-3, b bytes 4-7, c bytes 8-10 shifted up by 8 (:50-71)
    tail = data[i:]
    for k, byte in enumerate(tail):
        if k < 4:
            a = (a + (byte << (8 * k))) & M32
        elif k < 8:
            b = (b + (byte << (8 * (k - 4)))) & M32
        else:
            c = (c + (byte << (8 * (k - 8) + 8))) & M32
    a, b, c = _mix(a, b, c)
    return c


def jenkins_u64x3(u1: int, u2: int, u3: int) -> int:
    """JenkinsHash.ComputeHash(ulong,ulong,ulong), JenkinsHash.cs:85-105."""
    a = b = 0x9E3779B9
    c = 0
    a = (a + (u1 & M32)) & M32
    b = (b + (u1 >> 32)) & M32
    c = (c + (u2 & M32)) & M32
    a, b, c = _mix(a, b, c)
    a = (a + (u2 >> 32)) & M32
    b = (b + (u3 & M32)) & M32
    c = (c + (u3 >> 32)) & M32
    a, b, c = _mix(a, b, c)
    c = (c + 24) & M32
    a, b, c = _mix(a, b, c)
    return c


def _mix_np(a, b, c):
    a = a - b - c; a ^= c >> np.uint32(13)
    b = b - c - a; b ^= a << np.uint32(8)
    c = c - a - b; c ^= b >> np.uint32(13)
    a = a - b - c; a ^= c >> np.uint32(12)
    b = b - c - a; b ^= a << np.uint32(16)
    c = c - a - b; c ^= b >> np.uint32(5)
    a = a - b - c; a ^= c >> np.uint32(3)
    b = b - c - a; b ^= a << np.uint32(10)
    c = c - a - b; c ^= b >> np.uint32(15)
    return a, b, c


def jenkins_u64x3_np(u1: np.ndarray, u2: np.ndarray, u3: np.ndarray) -> np.ndarray:
    """Vectorised JenkinsHash.cs:85-105 over uint64 arrays -> uint32 array."""
    u1 = np.asarray(u1, dtype=np.uint64); u2 = np.asarray(u2, dtype=np.uint64)
    u3 = np.asarray(u3, dtype=np.uint64)
    lo = lambda x: (x & np.uint64(M32)).astype(np.uint32)
    hi = lambda x: (x >> np.uint64(32)).astype(np.uint32)
    with np.errstate(over="ignore"):
        a = np.full(u1.shape, 0x9E3779B9, dtype=np.uint32)
        b = a.copy()
        c = np.zeros(u1.shape, dtype=np.uint32)
        a = a + lo(u1); b = b + hi(u1); c = c + lo(u2)
        a, b, c = _mix_np(a, b, c)
        a = a + hi(u2); b = b + lo(u3); c = c + hi(u3)
        a, b, c = _mix_np(a, b, c)
        c = c + np.uint32(24)
        a, b, c = _mix_np(a, b, c)
    return c


# ---------------------------------------------------------------------------
# L0: UniqueKey / GrainId   src/Orleans.Core.Abstractions/IDs/{UniqueKey,GrainId}.cs
# ---------------------------------------------------------------------------


def type_code_data(category: int, type_data: int) -> int:
    """UniqueKey.NewKey(n0,n1,category,typeData,..), UniqueKey.cs:112-120:
    ``((ulong)category << 56) + ((ulong)typeData & 0x00FFFFFFFFFFFFFF)`` with
    typeData a C# long (sign-extended from the int grain type code)."""
    return ((category << 56) + ((type_data & M64) & 0x00FFFFFFFFFFFFFF)) & M64


def category_of(tcd: int) -> int:
    """UniqueKey.GetCategory, UniqueKey.cs:383-386."""
    return (tcd >> 56) & 0xFF


@dataclass(frozen=True)
class UniqueKey:
    """UniqueKey fields, UniqueKey.cs:28-31."""
    n0: int
    n1: int
    tcd: int
    key_ext: Optional[str] = None

    @property
    def category(self) -> int:
        return category_of(self.tcd)

    @property
    def has_key_ext(self) -> bool:
        return self.category in (CAT_KEYEXT_GRAIN, CAT_GEO_CLIENT)  # UniqueKey.cs:60-66

    def to_byte_array(self) -> bytes:
        """UniqueKey.ToByteArray, UniqueKey.cs:295-336 (== BinaryTokenStreamWriter
        Write(UniqueKey), BinaryTokenStreamWriter.cs:37-43)."""
        head = struct.pack("<QQQ", self.n0, self.n1, self.tcd)
        if self.key_ext is None:
            return head + struct.pack("<i", -1)
        ext = self.key_ext.encode("utf-8")
        return head + struct.pack("<i", len(ext)) + ext

    def uniform_hash(self) -> int:
        """UniqueKey.GetUniformHashCode, UniqueKey.cs:272-293.  Argument order is
        (TypeCodeData, N0, N1)."""
        if self.has_key_ext and self.key_ext is not None:
            return jenkins_bytes(self.to_byte_array())
        return jenkins_u64x3(self.tcd, self.n0, self.n1)

    def as_tuple(self) -> Tuple[int, int, int]:
        return (self.n0, self.n1, self.tcd)


def grain_id_long(type_code: int, primary_key: int) -> UniqueKey:
    """GrainId.GetGrainId(long typeCode, long primaryKey), GrainId.cs:72-77 ->
    UniqueKey.NewKey(long,..), UniqueKey.cs:122-128: N0 = 0, N1 = (ulong)key."""
    return UniqueKey(0, primary_key & M64, type_code_data(CAT_GRAIN, type_code))


def guid_key(guid: str, category: int, type_data: int = 0) -> UniqueKey:
    """UniqueKey.NewKey(Guid,..), UniqueKey.cs:135-143; Guid.ToByteArray is the
    mixed-endian layout that uuid.bytes_le reproduces."""
    b = uuid.UUID(guid).bytes_le
    n0, n1 = struct.unpack("<QQ", b)
    return UniqueKey(n0, n1, type_code_data(category, type_data))


# Constants.SystemMembershipTableId, src/Orleans.Core/Runtime/Constants.cs:52
MEMBERSHIP_TABLE_ID = guid_key("01145FEC-C21E-11E0-9105-D0FB4724019B", CAT_SYSTEM_GRAIN)


def calculate_id_hash(text: str) -> int:
    """Utils.CalculateIdHash, src/Orleans.Core/Utils/Utils.cs:184-203 (and the
    private copy SiloAddress.cs:176-195): SHA-256 over UTF-16LE, XOR of the 8
    big-endian int32 words, as a signed int32."""
    digest = hashlib.sha256(text.encode("utf-16-le")).digest()
    h = 0
    for i in range(0, 32, 4):
        h ^= int.from_bytes(digest[i:i + 4], "big")
    return h - (1 << 32) if h & 0x80000000 else h


def grain_type_code(full_type_name: str) -> int:
    """GrainInterfaceUtils.GetTypeCode, src/Orleans.Core/CodeGeneration/
    GrainInterfaceUtils.cs:400-415 (no [TypeCodeOverride], non-generic)."""
    return calculate_id_hash(full_type_name)


# ---------------------------------------------------------------------------
# L0: SiloAddress   src/Orleans.Core.Abstractions/IDs/SiloAddress.cs
# ---------------------------------------------------------------------------


@dataclass(frozen=True)
class Silo:
    ip: str
    port: int
    gen: int

    def endpoint_str(self) -> str:
        # IPEndPoint.ToString(): "a.b.c.d:port" / "[v6]:port" (canonical text of the parsed address;
        # the IPv6 form is an unpinned assumption)
        addr = ipaddress.ip_address(self.ip)
        if addr.version == 4:
            return f"{addr}:{self.port}"
        if addr.ipv4_mapped is not None:        # .NET prints mapped addresses as ::ffff:a.b.c.d
            return f"[::ffff:{addr.ipv4_mapped}]:{self.port}"
        return f"[{addr.compressed}]:{self.port}"

    def consistent_hash(self) -> int:
        """SiloAddress.GetConsistentHashCode, SiloAddress.cs:164-173:
        CalculateIdHash(Endpoint + Generation.ToString(Invariant))."""
        return calculate_id_hash(self.endpoint_str() + str(self.gen))

    def wire_bytes(self) -> bytes:
        """BinaryTokenStreamWriter.Write(SiloAddress), BinaryTokenStreamWriter.cs:
        485-513: 16 B address (IPv4: 12 zero bytes + 4) + port int32 + gen int32."""
        addr = ipaddress.ip_address(self.ip)
        ipb = (b"\x00" * 12 + addr.packed) if addr.version == 4 else addr.packed
        return ipb + struct.pack("<ii", self.port, self.gen)

    def uniform_hashes(self, n: int) -> List[int]:
        """SiloAddress.GetUniformHashCodesImpl, SiloAddress.cs:205-248."""
        base = self.wire_bytes()
        return [jenkins_bytes(base + struct.pack("<i", extra)) for extra in range(n)]

    def compare_to(self, other: "Silo") -> int:
        """SiloAddress.CompareTo, SiloAddress.cs:280-329: generation, port, then
        IP bytes (same family)."""
        if self.gen != other.gen:
            return -1 if self.gen < other.gen else 1
        if self.port != other.port:
            return -1 if self.port < other.port else 1
        a = ipaddress.ip_address(self.ip); b = ipaddress.ip_address(other.ip)
        if a.version != b.version:
            return -1 if a.version < b.version else 1
        pa, pb = a.packed, b.packed
        return (pa > pb) - (pa < pb)


def to_int32(x: int) -> int:
    x &= M32
    return x - (1 << 32) if x & 0x80000000 else x


# ---------------------------------------------------------------------------
# L3: rings
# ---------------------------------------------------------------------------


def ring_d_build(silos: Sequence[Silo]) -> List[int]:
    """LocalGrainDirectory.AddServer, LocalGrainDirectory.cs:284-309: insert at
    FindLastIndex(h < hash) + 1 (sorted by signed consistent hash; a newcomer
    goes *before* existing equal hashes).  Returns silo indices in ring order;
    silos are added in the given order."""
    ring: List[int] = []
    hashes = [s.consistent_hash() for s in silos]
    for idx in range(len(silos)):
        h = hashes[idx]
        last = -1
        for j, r in enumerate(ring):
            if hashes[r] < h:
                last = j
        ring.insert(last + 1, idx)
    return ring


def ring_d_lookup(ring_hashes: Sequence[int], key_hash: int) -> int:
    """LocalGrainDirectory.CalculateTargetSilo, LocalGrainDirectory.cs:477-545,
    with IsSiloNextInTheRing :1141-1144 (excludeMySelf false, as LocalLookup
    passes at :801): scan from the end for the first ring[i].hash <= (int)hash;
    none -> the last entry.  Returns the ring position."""
    h = to_int32(key_hash)
    n = len(ring_hashes)
    for i in range(n - 1, -1, -1):
        if ring_hashes[i] <= h:
            return i
    return n - 1


def ring_r_lookup(ring_hashes: Sequence[int], key: int) -> int:
    """ConsistentRingProvider.CalculateTargetSilo(uint), ConsistentRingProvider.cs:
    322-367 + IsSiloNextInTheRing :369-372: first i with (long)ring[i] >= (long)key
    (int vs uint promotes to long, so negative silo hashes never match); none ->
    ring[0].  The ring is built like mode D (AddServer :92-133)."""
    for i, h in enumerate(ring_hashes):
        if h >= key:
            return i
    return 0


def ring_v_build(silos: Sequence[Silo], buckets: int = 30) -> Tuple[List[int], List[int]]:
    """VirtualBucketsRingProvider.AddServer, VirtualBucketsRingProvider.cs:122-149:
    SortedDictionary<uint, SiloAddress>; a collision keeps the lesser
    SiloAddress.CompareTo.  Returns (points ascending uint, owner silo index)."""
    bmap: Dict[int, int] = {}
    for idx, s in enumerate(silos):
        for h in s.uniform_hashes(buckets):
            if h in bmap and s.compare_to(silos[bmap[h]]) > 0:
                continue
            bmap[h] = idx
    pts = sorted(bmap)
    return pts, [bmap[p] for p in pts]


def ring_v_lookup(points: Sequence[int], key: int) -> int:
    """VirtualBucketsRingProvider.CalculateTargetSilo, :257-293: first bucket with
    point >= key (uint), else bucket 0.  Returns the bucket position."""
    for i, p in enumerate(points):
        if p >= key:
            return i
    return 0


def in_range(begin: int, end: int, n: int) -> bool:
    """SingleRange.InRange, src/Orleans.Core/Runtime/RingRange.cs:72-81: (begin, end]."""
    if begin < end:
        return begin < n <= end
    return n > begin or n <= end


# numpy versions of the lookups (search-based, equal to the scans above)
def ring_d_lookup_np(ring_hashes: np.ndarray, key_hash: np.ndarray) -> np.ndarray:
    rh = np.asarray(ring_hashes, dtype=np.int64)
    h = key_hash.astype(np.uint32).view(np.int32).astype(np.int64)
    pos = np.searchsorted(rh, h, side="right") - 1
    return np.where(pos < 0, len(rh) - 1, pos)


def ring_r_lookup_np(ring_hashes: np.ndarray, key: np.ndarray) -> np.ndarray:
    rh = np.asarray(ring_hashes, dtype=np.int64)
    k = key.astype(np.uint32).astype(np.int64)
    pos = np.searchsorted(rh, k, side="left")
    return np.where(pos >= len(rh), 0, pos)


def ring_v_lookup_np(points: np.ndarray, key: np.ndarray) -> np.ndarray:
    p = np.asarray(points, dtype=np.int64)
    pos = np.searchsorted(p, key.astype(np.uint32).astype(np.int64), side="left")
    return np.where(pos >= len(p), 0, pos)


# ---------------------------------------------------------------------------
# L3: directory partition  src/Orleans.Runtime/GrainDirectory/GrainDirectoryPartition.cs
# ---------------------------------------------------------------------------


@dataclass
class DirectoryPartition:
    """Dictionary<GrainId, IGrainInfo> (GrainDirectoryPartition.cs:215) holding
    single-activation grains: value = (activation index, activation silo)."""
    data: Dict[Tuple[int, int, int], Tuple[int, int]] = field(default_factory=dict)

    def add_single_activation(self, key: Tuple[int, int, int], act: int, silo: int) -> Tuple[int, int, bool]:
        """AddSingleActivation, GrainDirectoryPartition.cs:304-326 with
        GrainInfo.AddSingleActivation :110-124: the first registration wins;
        later ones get the existing address back.  Returns (act, silo, inserted)."""
        if key in self.data:
            a, s = self.data[key]
            return a, s, False
        self.data[key] = (act, silo)
        return act, silo, True

    def remove_activation(self, key: Tuple[int, int, int], act: int) -> bool:
        """RemoveActivation, GrainDirectoryPartition.cs:335-363 (Force cause): drop
        the instance if the activation matches; the grain goes with its last
        instance."""
        cur = self.data.get(key)
        if cur is not None and cur[0] == act:
            del self.data[key]
            return True
        return False

    def remove_grain(self, key: Tuple[int, int, int]) -> bool:
        """RemoveGrain, GrainDirectoryPartition.cs:370-377."""
        return self.data.pop(key, None) is not None

    def lookup(self, key: Tuple[int, int, int]) -> Optional[Tuple[int, int]]:
        """LookUpActivations, GrainDirectoryPartition.cs:385-441 (all silos
        valid: static membership snapshot)."""
        return self.data.get(key)


# ---------------------------------------------------------------------------
# L4: addressing a batch (Dispatcher.AddressMessage -> LocalLookup)
# ---------------------------------------------------------------------------


@dataclass
class RingSpec:
    mode: str                 # "D", "R" or "V"
    points: List[int]         # ring values in ring order (int32 for D/R, uint32 for V)
    owners: List[int]         # silo index for each ring position


def ring_spec(silos: Sequence[Silo], mode: str = "D", buckets: int = 30) -> RingSpec:
    if mode in ("D", "R"):
        order = ring_d_build(silos)
        return RingSpec(mode, [silos[i].consistent_hash() for i in order], order)
    pts, own = ring_v_build(silos, buckets)
    return RingSpec("V", pts, own)


def ring_owner_np(spec: RingSpec, hashes: np.ndarray) -> np.ndarray:
    owners = np.asarray(spec.owners, dtype=np.int64)
    if spec.mode == "D":
        pos = ring_d_lookup_np(np.asarray(spec.points), hashes)
    elif spec.mode == "R":
        pos = ring_r_lookup_np(np.asarray(spec.points), hashes)
    else:
        pos = ring_v_lookup_np(np.asarray(spec.points), hashes)
    return owners[pos]


def route_batch(keys: np.ndarray, spec: RingSpec, directory: Dict[Tuple[int, int, int], Tuple[int, int]],
                my_silo: int = 0, seed_silo: int = 0):
    """Address a batch of messages (keys: (N,3) uint64 [n0, n1, tcd]).

    Follows Dispatcher.AddressMessage (src/Orleans.Runtime/Core/Dispatcher.cs:715-743)
    -> PlacementDirectorsManager / RandomPlacementDirector (single activation =>
    places[0], RandomPlacementDirector.cs:33-53) -> LocalGrainDirectory.LocalLookup
    (LocalGrainDirectory.cs:797-837) -> CalculateTargetSilo (:477-545) ->
    LookUpActivations.  Whole-node model: the owner partition is always
    consulted.

    Returns (status u8, silo u32, act u32, owner u32, hash u32)."""
    keys = np.asarray(keys, dtype=np.uint64).reshape(-1, 3)
    n = keys.shape[0]
    n0, n1, tcd = keys[:, 0], keys[:, 1], keys[:, 2]
    h = jenkins_u64x3_np(tcd, n0, n1)
    owner = ring_owner_np(spec, h).astype(np.uint32)
    cat = (tcd >> np.uint64(56)).astype(np.uint32)
    status = np.full(n, ST_OK, dtype=np.uint8)
    silo = owner.copy()
    act = np.full(n, M32, dtype=np.uint32)
    mt = MEMBERSHIP_TABLE_ID
    for i in range(n):
        c = int(cat[i])
        k = (int(n0[i]), int(n1[i]), int(tcd[i]))
        if c == CAT_SYSTEM_TARGET:                         # :480-485
            status[i] = ST_SYSTEM_TARGET; silo[i] = my_silo; owner[i] = my_silo
            continue
        if k == mt.as_tuple():                               # :487-503
            status[i] = ST_MEMBERSHIP; silo[i] = seed_silo; owner[i] = seed_silo
            continue
        if c in (CAT_KEYEXT_GRAIN, CAT_GEO_CLIENT):          # UniqueKey.cs:279-281
            status[i] = ST_KEYEXT; silo[i] = M32; owner[i] = M32
            continue
        v = directory.get(k)
        if v is None:
            status[i] = ST_MISS                               # Dispatcher.cs:742 slow path
        elif v[0] == ACT_MULTI:
            status[i] = ST_MULTI_ACT                          # RandomPlacementDirector.cs:33-53, in C#
        else:
            act[i], silo[i] = v
    return status, silo, act, owner, h


# ---------------------------------------------------------------------------
# L2/L4 receive: per-activation FIFO  (ActivationData.waiting, WorkItemGroup)
# ---------------------------------------------------------------------------


def bucket_stable(act: np.ndarray, n_act: int):
    """Per-activation enqueue order.  The reference appends each received
    message to its activation's FIFO in arrival order (IncomingMessageAgent.cs:
    92-190 -> WorkItemGroup.EnqueueTask, WorkItemGroup.cs:174-201 ->
    ActivationData.EnqueueMessage / waiting.Add, ActivationData.cs:566-606).
    A stable partition by activation reproduces exactly that.  Values >= n_act
    (unrouted messages) go to a trailing bucket n_act.

    Returns (perm u32[N], offsets u32[n_act + 2])."""
    a = np.asarray(act, dtype=np.uint64)
    a = np.minimum(a, np.uint64(n_act)).astype(np.int64)
    perm = np.argsort(a, kind="stable").astype(np.uint32)
    counts = np.bincount(a, minlength=n_act + 1)
    offsets = np.zeros(n_act + 2, dtype=np.uint32)
    offsets[1:] = np.cumsum(counts, dtype=np.uint64).astype(np.uint32)
    return perm, offsets


def bucket_fifo_loop(act: Sequence[int], n_act: int):
    """Pure-Python per-activation FIFO append (ActivationData.cs:604-605), small
    cases only; used to pin bucket_stable."""
    queues: List[List[int]] = [[] for _ in range(n_act + 1)]
    for i, a in enumerate(act):
        queues[min(int(a), n_act)].append(i)
    perm = [i for q in queues for i in q]
    offsets = [0]
    for q in queues:
        offsets.append(offsets[-1] + len(q))
    return np.asarray(perm, dtype=np.uint32), np.asarray(offsets, dtype=np.uint32)


# ---------------------------------------------------------------------------
# Synthetic workloads (SURVEY 8 d)
# ---------------------------------------------------------------------------

PING_GRAIN_CLASS = "BenchmarkGrains.Ping.PingGrain"


def bench_silos(n: int = 8) -> List[Silo]:
    """SiloAddress = 10.0.0.{1..S}:11111, generation 1 (SURVEY 8 d)."""
    return [Silo(f"10.0.0.{i + 1}", 11111, 1) for i in range(n)]


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def grain_keys(type_code: int, ks: np.ndarray) -> np.ndarray:
    """(N,3) uint64 [n0, n1, tcd] for GrainId.GetGrainId(typeCode, k)."""
    ks = np.asarray(ks, dtype=np.int64)
    out = np.zeros((ks.shape[0], 3), dtype=np.uint64)
    out[:, 1] = ks.view(np.uint64)
    out[:, 2] = np.uint64(type_code_data(CAT_GRAIN, type_code))
    return out


# ---------------------------------------------------------------------------
# vectorised batch addressing (same semantics as route_batch, for large N)
# ---------------------------------------------------------------------------


def _key_void(keys: np.ndarray) -> np.ndarray:
    k = np.ascontiguousarray(np.asarray(keys, dtype=np.uint64).reshape(-1, 3).astype(">u8"))
    return k.view("V24").ravel()


class DirectoryArrays:
    """Directory snapshot as sorted arrays (single-activation grains):
    key -> (act, silo).  Built from registrations applied in order, first wins
    (GrainDirectoryPartition.AddSingleActivation, :304-326)."""

    def __init__(self, keys: np.ndarray, acts: np.ndarray, silos: np.ndarray):
        kv = _key_void(keys)
        # first registration of each key wins
        uniq, first = np.unique(kv, return_index=True)
        self.sorted_keys = uniq
        self.acts = np.asarray(acts, dtype=np.uint32)[first]
        self.silos = np.asarray(silos, dtype=np.uint32)[first]

    def lookup(self, keys: np.ndarray):
        kv = _key_void(keys)
        if len(self.sorted_keys) == 0:
            z = np.zeros(len(kv), dtype=bool)
            return z, np.full(len(kv), M32, np.uint32), np.full(len(kv), M32, np.uint32)
        pos = np.searchsorted(self.sorted_keys, kv)
        pos_c = np.minimum(pos, len(self.sorted_keys) - 1)
        found = self.sorted_keys[pos_c] == kv
        act = np.where(found, self.acts[pos_c], M32).astype(np.uint32)
        silo = np.where(found, self.silos[pos_c], M32).astype(np.uint32)
        return found, act, silo


def directory_keys(d: DirectoryArrays) -> np.ndarray:
    """The (n,3) u64 keys of a DirectoryArrays snapshot (inverse of _key_void)."""
    if len(d.sorted_keys) == 0:
        return np.zeros((0, 3), dtype=np.uint64)
    return np.frombuffer(d.sorted_keys.tobytes(), dtype=">u8").reshape(-1, 3).astype(np.uint64)


def split_directory(d: DirectoryArrays, spec: RingSpec, keep, my_silo: int = 0, seed_silo: int = M32):
    """GrainDirectoryPartition.Split(grain => CalculateTargetSilo(grain) is not kept, true)
    (GrainDirectoryPartition.cs:532-570; predicate GrainDirectoryHandoffManager.cs:212-218).
    `keep` = silo indices held here.  KeyExt grains (owner needs the KeyExt string) stay.
    Returns (moved keys, acts, silos) sorted by key, and the remaining snapshot."""
    keys = directory_keys(d)
    st, silo, act, owner, h = route_batch_np(keys, spec, DirectoryArrays(np.zeros((0, 3), np.uint64), [], []),
                                             my_silo=my_silo, seed_silo=seed_silo)
    keep_set = np.zeros(max([int(x) for x in keep] + [int(owner[owner != M32].max()) if (owner != M32).any() else 0])
                        + 1, dtype=bool)
    keep_set[[int(x) for x in keep]] = True
    known = owner != M32
    sel = known & ~keep_set[np.where(known, owner, 0)]
    rest = DirectoryArrays(keys[~sel], d.acts[~sel], d.silos[~sel])
    return keys[sel], d.acts[sel], d.silos[sel], rest


def merge_directory(d: DirectoryArrays, keys, acts, silos):
    """GrainDirectoryPartition.Merge as a batched AddSingleActivation (first registration
    wins, existing entries first).  Returns (merged snapshot, inserted flags per incoming)."""
    keys = np.asarray(keys, dtype=np.uint64).reshape(-1, 3)
    found, _, _ = d.lookup(keys) if len(keys) else (np.zeros(0, bool), None, None)
    kv = _key_void(keys)
    _, first = np.unique(kv, return_index=True)
    first_mask = np.zeros(len(keys), dtype=bool)
    first_mask[first] = True
    inserted = ~found & first_mask
    merged = DirectoryArrays(np.concatenate([directory_keys(d), keys]), np.concatenate([d.acts, acts]),
                             np.concatenate([d.silos, silos]))
    return merged, inserted


def route_batch_np(keys: np.ndarray, spec: RingSpec, directory: DirectoryArrays,
                   my_silo: int = 0, seed_silo: int = M32):
    """Vectorised route_batch (Dispatcher.cs:715-743 -> LocalGrainDirectory.cs:
    477-545, 797-837 -> GrainDirectoryPartition.cs:385-441).
    Returns (status u8, silo u32, act u32, owner u32, hash u32)."""
    keys = np.asarray(keys, dtype=np.uint64).reshape(-1, 3)
    n0, n1, tcd = keys[:, 0], keys[:, 1], keys[:, 2]
    h = jenkins_u64x3_np(tcd, n0, n1)
    owner = ring_owner_np(spec, h).astype(np.uint32)
    cat = (tcd >> np.uint64(56)).astype(np.uint32)
    found, act, dsilo = directory.lookup(keys)
    status = np.where(found, ST_OK, ST_MISS).astype(np.uint8)
    silo = np.where(found, dsilo, owner).astype(np.uint32)
    # a grain with several activations (GrainInfo.Instances.Count >= 2): RandomPlacementDirector's
    # random choice (RandomPlacementDirector.cs:33-53) is left to C#; the silo is the owner's
    multi = found & (act == ACT_MULTI)
    status[multi] = ST_MULTI_ACT
    silo[multi] = owner[multi]
    act = np.where(multi, M32, act).astype(np.uint32)
    mt = MEMBERSHIP_TABLE_ID
    is_mt = (n0 == np.uint64(mt.n0)) & (n1 == np.uint64(mt.n1)) & (tcd == np.uint64(mt.tcd))
    is_st = cat == CAT_SYSTEM_TARGET
    is_ke = (cat == CAT_KEYEXT_GRAIN) | (cat == CAT_GEO_CLIENT)
    # precedence: system target, then membership grain, then KeyExt (LocalGrainDirectory.cs:480-503)
    ke = is_ke & ~is_st & ~is_mt
    mtm = is_mt & ~is_st
    status[ke] = ST_KEYEXT; silo[ke] = M32; owner[ke] = M32; act[ke] = M32
    status[mtm] = ST_MEMBERSHIP; silo[mtm] = seed_silo; owner[mtm] = seed_silo; act[mtm] = M32
    status[is_st] = ST_SYSTEM_TARGET; silo[is_st] = my_silo; owner[is_st] = my_silo; act[is_st] = M32
    return status, silo, act, owner, h


def fmix32_np(h: np.ndarray) -> np.ndarray:
    """MurmurHash3's 32-bit finaliser, vectorised (the table's home-slot mix, gd_common.h fmix32)."""
    h = np.asarray(h, dtype=np.uint64) & np.uint64(M32)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & np.uint64(M32)
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & np.uint64(M32)
    h ^= h >> np.uint64(16)
    return h.astype(np.uint32)


N_REGIONS = 8


def table_region_np(keys: np.ndarray) -> np.ndarray:
    """The owner's table region of each message (not a reference concept: the library's exchange
    order): the top 3 bits of fmix32(uniform hash) for a grain the owner probes in its
    directory table -- the eighth of the table its home slot falls in -- and 0 for system targets,
    the membership grain and KeyExt / geo-client grains (LocalGrainDirectory.cs:480-503 route
    those without the table)."""
    keys = np.asarray(keys, dtype=np.uint64).reshape(-1, 3)
    n0, n1, tcd = keys[:, 0], keys[:, 1], keys[:, 2]
    cat = (tcd >> np.uint64(56)).astype(np.uint32)
    mt = MEMBERSHIP_TABLE_ID
    special = ((cat == CAT_SYSTEM_TARGET) | (cat == CAT_KEYEXT_GRAIN) | (cat == CAT_GEO_CLIENT) |
               ((n0 == np.uint64(mt.n0)) & (n1 == np.uint64(mt.n1)) & (tcd == np.uint64(mt.tcd))))
    reg = fmix32_np(jenkins_u64x3_np(tcd, n0, n1)) >> np.uint32(32 - 3)
    return np.where(special, 0, reg).astype(np.uint32)


def region_order(keys: np.ndarray) -> np.ndarray:
    """Positions of one sender's chunk in the order the owner receives them from gd_route_multi:
    stable by table region (table_region_np), batch order within a region."""
    return np.argsort(table_region_np(keys), kind="stable")
