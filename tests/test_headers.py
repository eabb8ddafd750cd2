"""SURVEY 8 f1 oracle tests (CPU): Orleans message frame / header wire format.

The reference's own coverage of this format is MessageSerializerTests.MessageTest_BinaryRoundTrip
(test/NonSilo.Tests/Serialization/MessageSerializerTests.cs:30-125): a runtime round trip with
no byte fixtures.  Here the oracle is pinned by (1) a frame assembled byte-by-byte from the
writer's field encodings, independent of oracle.headers.encode_headers, carrying the same
headers that test sets; (2) the frozen golden frames; (3) round trips and edge cases.
"""
import json
import os
import struct
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "oracle"))
import headers as H  # noqa: E402
import oracle as o  # noqa: E402

GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))


LOOPBACK_IP = bytes(12) + bytes([127, 0, 0, 1])


def _loopback(port, gen=0):
    # BinaryTokenStreamWriter.Write(IPAddress): IPv4 -> 12 zero bytes + 4 address bytes (:491-505)
    return LOOPBACK_IP + struct.pack("<ii", port, gen)


def test_header_mask_bits_match_reference_enum():
    # HeadersContainer.Headers (Message.cs:728-765)
    assert [H.ALWAYS_INTERLEAVE, H.CACHE_INVALIDATION_HEADER, H.CATEGORY, H.CORRELATION_ID] == [1, 2, 4, 8]
    assert H.SENDING_ACTIVATION == 1 << 15 and H.TARGET_GRAIN == 1 << 20 and H.TARGET_SILO == 1 << 21
    assert H.REQUEST_CONTEXT == 1 << 24 and H.TRANSACTION_INFO == 1 << 27 and H.IS_TRANSACTION_REQUIRED == 1 << 28
    assert (H.TRUE_TOKEN, H.FALSE_TOKEN) == (3, 4)          # SerializationTokenType.cs:10-11


def test_known_answer_frame_binary_round_trip_message():
    """The headers MessageTest_BinaryRoundTrip sets (MessageSerializerTests.cs:73-81), assembled by hand."""
    tcd = o.type_code_data(o.CAT_GRAIN, 1234)
    sending, target = (11, 12, tcd), (21, 22, tcd)
    corr = 0x0102030405060708
    mask = (H.CATEGORY | H.DIRECTION | H.CORRELATION_ID | H.ALWAYS_INTERLEAVE | H.SENDING_GRAIN |
            H.SENDING_SILO | H.TARGET_GRAIN | H.TARGET_SILO | H.IS_USING_INTERFACE_VERSION)
    want = (struct.pack("<I", mask) + bytes([2])            # Category = Application
            + bytes([0])                                     # Direction = Request
            + corr.to_bytes(8, "little")                     # CorrelationId: BitConverter bytes
            + bytes([3])                                     # IsAlwaysInterleave: True token
            + struct.pack("<QQQi", *sending, -1)             # SendingGrain, KeyExt null
            + _loopback(200)                                 # SendingSilo
            + struct.pack("<QQQi", *target, -1)              # TargetGrain
            + _loopback(300))                                # TargetSilo
    assert len(want) == 4 + 1 + 1 + 8 + 1 + 28 + 24 + 28 + 24
    hdr = H.encode_headers({"category": 2, "direction": 0, "correlation_id": corr, "always_interleave": True,
                            "sending_grain": (sending, None), "sending_silo": (LOOPBACK_IP, 200, 0),
                            "target_grain": (target, None), "target_silo": (LOOPBACK_IP, 300, 0),
                            "is_using_interface_version": True})
    assert hdr == want
    body = b"\x01\x02\x03"
    frame = struct.pack("<ii", len(want), len(body)) + want + body    # Message.cs:481-516
    r = H.decode_frame(frame, 0)
    assert r["flags"] == H.F_HAS_TARGET                               # no TargetActivation -> not complete
    assert r["target_grain"] == target and r["sending_grain"] == sending
    assert r["category"] == 2 and r["direction"] == 0 and r["correlation_id"] == corr
    assert r["target_silo"] == _loopback(300) and r["sending_silo"] == _loopback(200)
    assert r["mask"] == mask


def test_golden_frames_pin_oracle():
    g = GOLDEN["frames"]
    buf = bytes.fromhex(g["buffer_hex"])
    dec = H.decode_frames(buf, g["offsets"])
    assert dec["flags"].tolist() == g["flags"] and dec["mask"].tolist() == g["mask"]
    assert [[str(int(x)) for x in k] for k in dec["target_grain"]] == g["target_grain"]
    assert [[str(int(x)) for x in k] for k in dec["sending_grain"]] == g["sending_grain"]
    assert [bytes(x).hex() for x in dec["target_silo"]] == g["target_silo_hex"]
    assert [str(int(x)) for x in dec["correlation_id"]] == g["correlation_id"]
    assert dec["category"].tolist() == g["category"] and dec["direction"].tolist() == g["direction"]
    # every flag class is represented
    fl = set(g["flags"])
    assert H.F_MALFORMED in fl and any(f & H.F_FALLBACK for f in fl) and any(f & H.F_COMPLETE for f in fl)


def test_random_round_trip():
    rng = np.random.default_rng(7)
    keys = o.grain_keys(o.grain_type_code(o.PING_GRAIN_CLASS), rng.integers(0, 1 << 20, size=3000))
    buf, offs = H.random_frames(3000, keys, rng, p_fallback=0.0, p_complete=0.1, p_malformed=0.0)
    dec = H.decode_frames(buf, offs)
    ok = (dec["flags"] & H.F_HAS_TARGET) != 0
    obs = (dec["mask"] & H.TARGET_OBSERVER) != 0
    assert ok.all()
    assert np.array_equal(dec["target_grain"], keys)
    # only observer + target-silo frames fall back (TargetObserver is object-serialized)
    fb = (dec["flags"] & H.F_FALLBACK) != 0
    assert np.array_equal(fb, obs & ((dec["mask"] & H.TARGET_SILO) != 0))
    assert np.array_equal((dec["flags"] & H.F_COMPLETE) != 0,
                          (dec["mask"] & (H.TARGET_ACTIVATION | H.TARGET_SILO | H.TARGET_GRAIN)) ==
                          (H.TARGET_ACTIVATION | H.TARGET_SILO | H.TARGET_GRAIN))


@pytest.mark.parametrize("case", ["short_buffer", "hl_small", "neg_body", "body_past_end", "bad_string",
                                  "string_past_header", "empty_batch", "cache_invalidation", "key_ext"])
def test_edge_cases(case):
    k = (1, 2, o.type_code_data(o.CAT_GRAIN, 9))
    good = H.encode_frame({"target_grain": (k, None), "debug_context": "dbg"})
    if case == "short_buffer":
        assert H.decode_frame(good[:7], 0)["flags"] == H.F_MALFORMED
    elif case == "hl_small":
        f = struct.pack("<ii", 3, 0) + b"\0" * 3
        assert H.decode_frame(f, 0)["flags"] == H.F_MALFORMED
    elif case == "neg_body":
        f = bytearray(good); struct.pack_into("<i", f, 4, -1)
        assert H.decode_frame(bytes(f), 0)["flags"] == H.F_MALFORMED
    elif case == "body_past_end":
        f = bytearray(good); struct.pack_into("<i", f, 4, 1)
        assert H.decode_frame(bytes(f), 0)["flags"] == H.F_MALFORMED
    elif case == "bad_string":
        f = bytearray(good); struct.pack_into("<i", f, 12, -2)           # DebugContext length < -1
        assert H.decode_frame(bytes(f), 0)["flags"] == H.F_MALFORMED
    elif case == "string_past_header":
        f = bytearray(good); struct.pack_into("<i", f, 12, 1000)
        r = H.decode_frame(bytes(f), 0)
        assert r["flags"] == H.F_MALFORMED and r["target_grain"] == (0, 0, 0) and r["mask"] == 0
    elif case == "empty_batch":
        d = H.decode_frames(b"", np.zeros(0, dtype=np.uint64))
        assert d["flags"].shape == (0,) and d["target_grain"].shape == (0, 3)
    elif case == "cache_invalidation":
        f = H.encode_frame({"cache_invalidation": struct.pack("<i", 0), "target_grain": (k, None)})
        r = H.decode_frame(f, 0)
        assert r["flags"] == H.F_FALLBACK and r["target_grain"] == (0, 0, 0)
    elif case == "key_ext":
        f = H.encode_frame({"target_grain": (k, "ext-é"), "category": 1})
        r = H.decode_frame(f, 0)
        assert r["flags"] == H.F_HAS_TARGET | H.F_TARGET_KEYEXT and r["target_grain"] == k and r["category"] == 1


def test_route_frames_status_patch():
    g = GOLDEN["frames"]
    st = np.array(g["route_status"])
    fl = np.array(g["flags"])
    undecoded = ((fl & H.F_HAS_TARGET) == 0) | ((fl & (H.F_FALLBACK | H.F_MALFORMED)) != 0)
    assert (st[undecoded] == H.ROUTE_UNDECODED).all()
    assert (st[~undecoded & ((fl & H.F_COMPLETE) != 0)] == H.ROUTE_ADDRESSED).all()
    assert (np.array(g["route_act"])[st >= H.ROUTE_ADDRESSED] == 0xFFFFFFFF).all()
