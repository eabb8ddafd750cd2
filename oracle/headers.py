"""Oracle for SURVEY 8 f1: Orleans message frames and header decode -- TEST
INFRASTRUCTURE ONLY (checker for libgraindispatch's gd_decode_frames*).

Restates, from the C# source text:
  * the frame: [int32 headerLength][int32 bodyLength][header bytes][body bytes]
    (Message.Serialize, src/Orleans.Core/Messaging/Message.cs:481-516);
  * the header: int32 mask (HeadersContainer.Headers, Message.cs:728-765), then
    the present fields in the order HeadersContainer.Serializer writes them
    (Message.cs:1126-1245);
  * field encodings (src/Orleans.Core/Serialization/BinaryTokenStreamWriter.cs):
    byte / int32 / int64 little-endian; bool = 1 token byte; string = int32
    UTF-8 length (-1 = null) + bytes (:280-293); TimeSpan = ticks int64 (:516-519);
    CorrelationId = 8 bytes (:22-25, CorrelationId.cs:94-97); UniqueKey
    (GrainId / ActivationId) = N0, N1, TypeCodeData u64 + KeyExt string (:37-57);
    SiloAddress = 16-byte IP + int32 port + int32 generation (:485-513).
Fields that go through the C# object serializer (CacheInvalidationHeader,
RequestContext, TargetObserver, TransactionInfo) are written here as opaque
byte runs; a decoder cannot size them without that serializer, so a frame with
one of them BEFORE TargetGrain is a fallback frame.
"""
import struct
from typing import Dict, List, Optional, Tuple

import numpy as np

# HeadersContainer.Headers bits (Message.cs:728-765)
ALWAYS_INTERLEAVE = 1 << 0
CACHE_INVALIDATION_HEADER = 1 << 1
CATEGORY = 1 << 2
CORRELATION_ID = 1 << 3
DEBUG_CONTEXT = 1 << 4
DIRECTION = 1 << 5
TIME_TO_LIVE = 1 << 6
FORWARD_COUNT = 1 << 7
NEW_GRAIN_TYPE = 1 << 8
GENERIC_GRAIN_TYPE = 1 << 9
RESULT = 1 << 10
REJECTION_INFO = 1 << 11
REJECTION_TYPE = 1 << 12
READ_ONLY = 1 << 13
RESEND_COUNT = 1 << 14
SENDING_ACTIVATION = 1 << 15
SENDING_GRAIN = 1 << 16
SENDING_SILO = 1 << 17
IS_NEW_PLACEMENT = 1 << 18
TARGET_ACTIVATION = 1 << 19
TARGET_GRAIN = 1 << 20
TARGET_SILO = 1 << 21
TARGET_OBSERVER = 1 << 22
IS_UNORDERED = 1 << 23
REQUEST_CONTEXT = 1 << 24
IS_RETURNED_FROM_REMOTE_CLUSTER = 1 << 25
IS_USING_INTERFACE_VERSION = 1 << 26
TRANSACTION_INFO = 1 << 27
IS_TRANSACTION_REQUIRED = 1 << 28

# frame flags reported by the decoder (include/graindispatch.h GD_FRAME_*)
F_HAS_TARGET, F_COMPLETE, F_FALLBACK, F_MALFORMED = 1, 2, 4, 8

TRUE_TOKEN, FALSE_TOKEN = 3, 4     # SerializationTokenType.True / False (SerializationTokenType.cs:10-11)


def w_string(s: Optional[str]) -> bytes:
    if s is None:
        return struct.pack("<i", -1)
    b = s.encode("utf-8")
    return struct.pack("<i", len(b)) + b


def w_key(k: Tuple[int, int, int], ext: Optional[str] = None) -> bytes:
    return struct.pack("<QQQ", *k) + w_string(ext)


def w_silo(ip16: bytes, port: int, gen: int) -> bytes:
    return ip16 + struct.pack("<ii", port, gen)


def encode_headers(h: Dict) -> bytes:
    """HeadersContainer.Serializer (Message.cs:1126-1245).  `h` maps field names to
    values; a present key sets its mask bit.  Opaque object fields take raw bytes."""
    m = 0
    out = b""
    def has(name, bit):
        nonlocal m
        if name in h:
            m |= bit
            return True
        return False
    body = []
    if has("cache_invalidation", CACHE_INVALIDATION_HEADER):
        body.append(h["cache_invalidation"])                       # int count + WriteObj(...) -- opaque
    if has("category", CATEGORY):
        body.append(struct.pack("<B", h["category"]))
    if has("debug_context", DEBUG_CONTEXT):
        body.append(w_string(h["debug_context"]))
    if has("direction", DIRECTION):
        body.append(struct.pack("<B", h["direction"]))
    if has("time_to_live", TIME_TO_LIVE):
        body.append(struct.pack("<q", h["time_to_live"]))
    if has("forward_count", FORWARD_COUNT):
        body.append(struct.pack("<i", h["forward_count"]))
    if has("generic_grain_type", GENERIC_GRAIN_TYPE):
        body.append(w_string(h["generic_grain_type"]))
    if has("correlation_id", CORRELATION_ID):
        body.append(struct.pack("<q", h["correlation_id"]))
    if has("always_interleave", ALWAYS_INTERLEAVE):
        body.append(bytes([TRUE_TOKEN if h["always_interleave"] else FALSE_TOKEN]))
    if has("is_new_placement", IS_NEW_PLACEMENT):
        body.append(bytes([TRUE_TOKEN if h["is_new_placement"] else FALSE_TOKEN]))
    if has("read_only", READ_ONLY):
        body.append(bytes([TRUE_TOKEN if h["read_only"] else FALSE_TOKEN]))
    if has("is_unordered", IS_UNORDERED):
        body.append(bytes([TRUE_TOKEN if h["is_unordered"] else FALSE_TOKEN]))
    if has("new_grain_type", NEW_GRAIN_TYPE):
        body.append(w_string(h["new_grain_type"]))
    if has("rejection_info", REJECTION_INFO):
        body.append(w_string(h["rejection_info"]))
    if has("rejection_type", REJECTION_TYPE):
        body.append(struct.pack("<B", h["rejection_type"]))
    if has("request_context", REQUEST_CONTEXT):
        body.append(h["request_context"])                          # opaque
    if has("resend_count", RESEND_COUNT):
        body.append(struct.pack("<i", h["resend_count"]))
    if has("result", RESULT):
        body.append(struct.pack("<B", h["result"]))
    if has("sending_activation", SENDING_ACTIVATION):
        body.append(w_key(*h["sending_activation"]))
    if has("sending_grain", SENDING_GRAIN):
        body.append(w_key(*h["sending_grain"]))
    if has("sending_silo", SENDING_SILO):
        body.append(w_silo(*h["sending_silo"]))
    if has("target_activation", TARGET_ACTIVATION):
        body.append(w_key(*h["target_activation"]))
    if has("target_grain", TARGET_GRAIN):
        body.append(w_key(*h["target_grain"]))
    if has("target_observer", TARGET_OBSERVER):
        body.append(h["target_observer"])                          # opaque
    if has("target_silo", TARGET_SILO):
        body.append(w_silo(*h["target_silo"]))
    if has("transaction_info", TRANSACTION_INFO):
        body.append(h["transaction_info"])                         # opaque
    if h.get("is_using_interface_version"):
        m |= IS_USING_INTERFACE_VERSION                             # mask bit only (:1170-1171)
    return struct.pack("<i", m) + b"".join(body)


def encode_frame(h: Dict, body: bytes = b"") -> bytes:
    """Message.Serialize framing (Message.cs:481-516)."""
    hdr = encode_headers(h)
    return struct.pack("<ii", len(hdr), len(body)) + hdr + body


F_TARGET_KEYEXT = 16
FIELDS_DEFAULT = {"target_grain": (0, 0, 0), "target_activation": (0, 0, 0), "sending_activation": (0, 0, 0),
                  "sending_grain": (0, 0, 0), "target_silo": b"\0" * 24, "sending_silo": b"\0" * 24,
                  "correlation_id": 0, "category": 0, "direction": 0xFF, "mask": 0,
                  "target_ext": None}   # TargetGrain's KeyExt bytes (None: null or not decoded)


def decode_frame(buf: bytes, off: int):
    """Walk one frame's header (HeadersContainer.Deserializer, Message.cs:1247-1356)
    through TargetSilo, extracting the fields the dispatch path reads.

    flags: F_HAS_TARGET (TargetGrain decoded), F_COMPLETE (TargetGrain, TargetActivation
    and TargetSilo bits all set = TargetAddress.IsComplete, Message.cs:169-209 -- AddressMessage
    skips such a message, Dispatcher.cs:718), F_FALLBACK (an object-serialized field precedes a
    field read here: CacheInvalidationHeader / RequestContext before TargetGrain -> nothing is
    decoded; TargetObserver before TargetSilo -> everything but TargetSilo is decoded),
    F_MALFORMED (lengths run past the header or the buffer -> nothing decoded, mask 0),
    F_TARGET_KEYEXT (TargetGrain carries a KeyExt string).
    Absent fields keep FIELDS_DEFAULT (direction 0xFF = null)."""
    r = dict(FIELDS_DEFAULT)
    r["flags"] = 0
    n = len(buf)
    if off + 8 > n:
        r["flags"] = F_MALFORMED
        return r
    hl, bl = struct.unpack_from("<ii", buf, off)
    if hl < 4 or bl < 0 or off + 8 + hl + bl > n:
        r["flags"] = F_MALFORMED
        return r
    p, end = off + 12, off + 8 + hl
    m = struct.unpack_from("<I", buf, off + 8)[0]
    out = dict(FIELDS_DEFAULT)
    out["mask"] = m
    flags = F_COMPLETE if (m & TARGET_ACTIVATION and m & TARGET_SILO and m & TARGET_GRAIN) else 0
    if m & (CACHE_INVALIDATION_HEADER | REQUEST_CONTEXT):
        out["flags"] = flags | F_FALLBACK
        return out

    class Bad(Exception):
        pass

    def take(k):
        nonlocal p
        if p + k > end:
            raise Bad()
        b = buf[p:p + k]
        p += k
        return b

    def skip_string():
        ln = struct.unpack("<i", take(4))[0]
        if ln < -1:
            raise Bad()
        if ln > 0:
            take(ln)
        return ln

    def key():
        k = struct.unpack("<QQQ", take(24))
        return k, skip_string()

    def key_with_ext():
        """ReadUniqueKey keeping the KeyExt bytes (BinaryTokenStreamReader.cs:36-43)."""
        k = struct.unpack("<QQQ", take(24))
        ln = struct.unpack("<i", take(4))[0]
        if ln < -1:
            raise Bad()
        return k, ln, (take(ln) if ln > 0 else (b"" if ln == 0 else None))

    try:
        if m & CATEGORY:
            out["category"] = take(1)[0]
        if m & DEBUG_CONTEXT:
            skip_string()
        if m & DIRECTION:
            out["direction"] = take(1)[0]
        if m & TIME_TO_LIVE:
            take(8)
        if m & FORWARD_COUNT:
            take(4)
        if m & GENERIC_GRAIN_TYPE:
            skip_string()
        if m & CORRELATION_ID:
            out["correlation_id"] = struct.unpack("<q", take(8))[0]
        for bit in (ALWAYS_INTERLEAVE, IS_NEW_PLACEMENT, READ_ONLY, IS_UNORDERED):
            if m & bit:
                take(1)
        for bit in (NEW_GRAIN_TYPE, REJECTION_INFO):
            if m & bit:
                skip_string()
        if m & REJECTION_TYPE:
            take(1)
        if m & RESEND_COUNT:
            take(4)
        if m & RESULT:
            take(1)
        if m & SENDING_ACTIVATION:
            out["sending_activation"] = key()[0]
        if m & SENDING_GRAIN:
            out["sending_grain"] = key()[0]
        if m & SENDING_SILO:
            out["sending_silo"] = take(24)
        if m & TARGET_ACTIVATION:
            out["target_activation"] = key()[0]
        if m & TARGET_GRAIN:
            k, ext, ext_bytes = key_with_ext()
            out["target_grain"] = k
            out["target_ext"] = ext_bytes
            flags |= F_HAS_TARGET | (F_TARGET_KEYEXT if ext >= 0 else 0)
        if m & TARGET_SILO:
            if m & TARGET_OBSERVER:
                flags |= F_FALLBACK
            else:
                out["target_silo"] = take(24)
    except Bad:
        r["flags"] = F_MALFORMED
        return r
    out["flags"] = flags
    return out


def decode_frames(buf: bytes, offsets) -> Dict[str, np.ndarray]:
    """Vector form of decode_frame: one SoA array per field (the gd_frame_fields layout)."""
    rows = [decode_frame(buf, int(o)) for o in offsets]
    n = len(rows)
    def keys(name):
        return np.array([x[name] for x in rows], dtype=np.uint64).reshape(n, 3)
    def silos(name):
        return np.frombuffer(b"".join(x[name] for x in rows), dtype=np.uint8).reshape(n, 24)
    return {"flags": np.array([x["flags"] for x in rows], dtype=np.uint32),
            "mask": np.array([x["mask"] for x in rows], dtype=np.uint32),
            "target_grain": keys("target_grain"), "target_activation": keys("target_activation"),
            "sending_activation": keys("sending_activation"), "sending_grain": keys("sending_grain"),
            "target_silo": silos("target_silo"), "sending_silo": silos("sending_silo"),
            "correlation_id": np.array([x["correlation_id"] for x in rows], dtype=np.int64),
            "category": np.array([x["category"] for x in rows], dtype=np.uint8),
            "direction": np.array([x["direction"] for x in rows], dtype=np.uint8)}


# route statuses added by gd_route_frames (include/graindispatch.h)
ROUTE_ADDRESSED, ROUTE_UNDECODED = 5, 6


def route_frames_np(buf: bytes, offsets, spec, d):
    """Decode -> route -> status patch (SURVEY 8 f1 + a13): frames whose address is complete
    are not looked up (Dispatcher.cs:718) -> ADDRESSED; frames without a decoded TargetGrain
    (absent, fallback, malformed) -> UNDECODED; both carry no silo/activation."""
    import oracle as o
    f = decode_frames(buf, offsets)
    st, silo, act = o.route_batch_np(f["target_grain"], spec, d)[:3]
    st, silo, act = st.copy(), silo.copy(), act.copy()
    undecoded = ((f["flags"] & F_HAS_TARGET) == 0) | ((f["flags"] & (F_FALLBACK | F_MALFORMED)) != 0)
    addressed = ~undecoded & ((f["flags"] & F_COMPLETE) != 0)
    st[addressed] = ROUTE_ADDRESSED
    st[undecoded] = ROUTE_UNDECODED
    silo[addressed | undecoded] = 0xFFFFFFFF
    act[addressed | undecoded] = 0xFFFFFFFF
    return f, st, silo, act


def route_frames_ext_np(buf: bytes, offsets, spec, d, kxdir):
    """route_frames_np with KeyExt targets routed too (gd_route_frames_ext): the TargetGrain's
    KeyExt string comes from the frame itself (oracle/keyext.py route_batch_ext)."""
    import keyext as kx
    rows = [decode_frame(buf, int(o)) for o in offsets]
    f = decode_frames(buf, offsets)
    exts = [r.get("target_ext") for r in rows]
    st, silo, act = kx.route_batch_ext(f["target_grain"], exts, spec, d, kxdir)[:3]
    st, silo, act = st.copy(), silo.copy(), act.copy()
    undecoded = ((f["flags"] & F_HAS_TARGET) == 0) | ((f["flags"] & (F_FALLBACK | F_MALFORMED)) != 0)
    addressed = ~undecoded & ((f["flags"] & F_COMPLETE) != 0)
    st[addressed] = ROUTE_ADDRESSED
    st[undecoded] = ROUTE_UNDECODED
    silo[addressed | undecoded] = 0xFFFFFFFF
    act[addressed | undecoded] = 0xFFFFFFFF
    return f, st, silo, act


def random_frames(n: int, target_keys: np.ndarray, rng: np.random.Generator, p_fallback=0.03,
                  p_complete=0.05, p_malformed=0.01, target_exts=None):
    """Synthetic request frames around the given target GrainIds, with every optional
    field drawn at random.  target_exts[i] (str or None), when given, is frame i's TargetGrain
    KeyExt.  Returns (buffer bytes, frame offsets u64)."""
    parts, offs, pos = [], [], 0
    silo = (b"\x00" * 12 + bytes([10, 0, 0, 1]), 11111, 7)
    for i in range(n):
        h = {"category": 2, "direction": int(rng.integers(0, 3)), "correlation_id": int(rng.integers(1, 1 << 62))}
        k = tuple(int(x) for x in target_keys[i])
        ext_draw = "ext" if rng.random() < 0.02 else None
        h["target_grain"] = (k, target_exts[i] if target_exts is not None else ext_draw)
        if rng.random() < 0.5:
            h["sending_grain"] = ((0, int(rng.integers(0, 1 << 40)), int(target_keys[i][2])), None)
            h["sending_activation"] = ((int(rng.integers(1, 1 << 60)), int(rng.integers(0, 1 << 60)), 0), None)
            h["sending_silo"] = silo
        if rng.random() < 0.2:
            h["debug_context"] = "x" * int(rng.integers(0, 40))
        if rng.random() < 0.1:
            h["time_to_live"] = int(rng.integers(0, 1 << 40))
        if rng.random() < 0.1:
            h["forward_count"] = int(rng.integers(0, 3))
        if rng.random() < 0.1:
            h["generic_grain_type"] = None if rng.random() < 0.5 else "[[System.Int32]]"
        for f in ("always_interleave", "is_new_placement", "read_only", "is_unordered"):
            if rng.random() < 0.1:
                h[f] = bool(rng.random() < 0.5)
        if rng.random() < 0.05:
            h["new_grain_type"] = "Grains.Ping"
        if rng.random() < 0.05:
            h["resend_count"] = 1
        if rng.random() < p_complete:
            h["target_activation"] = ((int(rng.integers(1, 1 << 60)), 5, 0), None)
            h["target_silo"] = silo
        if rng.random() < 0.05:
            h["target_observer"] = bytes(rng.integers(0, 256, size=20, dtype=np.uint8))
        if rng.random() < p_fallback:
            h["request_context"] = struct.pack("<i", 1) + bytes(rng.integers(0, 256, size=30, dtype=np.uint8))
        body = bytes(rng.integers(0, 256, size=int(rng.integers(0, 64)), dtype=np.uint8))
        fr = bytearray(encode_frame(h, body))
        if rng.random() < p_malformed:       # truncate the header length: the walk runs off its end
            hl = struct.unpack_from("<i", fr, 0)[0]
            struct.pack_into("<i", fr, 0, max(4, hl - 20))
        parts.append(bytes(fr))
        offs.append(pos)
        pos += len(fr)
    return b"".join(parts), np.array(offs, dtype=np.uint64)
