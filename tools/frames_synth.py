"""Synthetic Orleans request frames at full size (numpy, vectorised) for the f1 decode bench
and the full-size GPU property test.  Input generation only -- the checker is oracle/headers.py.

Every frame carries the headers a grain-to-grain request has after MessageFactory.CreateMessage
+ Dispatcher.SendMessage (Message.cs:105-330; MessageFactory.cs:21-46): Category, Direction,
CorrelationId, SendingActivation, SendingGrain, SendingSilo, TargetGrain -- target not yet
addressed, so the frame goes through AddressMessage.  Layout (little-endian, BinaryTokenStreamWriter):

  [int32 hl][int32 bl] | mask | cat u8 | dir u8 | corr i64 | SendingActivation 24+4 |
  SendingGrain 24+4 | SendingSilo 24 | TargetGrain 24+4 | body (bl bytes)

hl = 122; with the default 40-byte body a frame is 170 bytes, so frames start on 2-byte
boundaries and every 4th one is dword aligned (the decoder handles any alignment).
"""
import numpy as np

CATEGORY, CORRELATION_ID, DIRECTION = 1 << 2, 1 << 3, 1 << 5
SENDING_ACTIVATION, SENDING_GRAIN, SENDING_SILO, TARGET_GRAIN = 1 << 15, 1 << 16, 1 << 17, 1 << 20
MASK = CATEGORY | CORRELATION_ID | DIRECTION | SENDING_ACTIVATION | SENDING_GRAIN | SENDING_SILO | TARGET_GRAIN
HEADER_LEN = 4 + 1 + 1 + 8 + 28 + 28 + 24 + 28


def build_frames(target_keys: np.ndarray, rng: np.random.Generator, body_len: int = 40,
                 sender_keys: np.ndarray = None):
    """Returns (buffer uint8[n * frame_len], offsets uint64[n], frame_len)."""
    tk = np.ascontiguousarray(np.asarray(target_keys, dtype=np.uint64).reshape(-1, 3))
    n = len(tk)
    fl = 8 + HEADER_LEN + body_len
    rec = np.zeros((n, fl), dtype=np.uint8)

    def put(col, arr):
        a = np.ascontiguousarray(arr)
        b = a.view(np.uint8).reshape(n, -1)
        rec[:, col:col + b.shape[1]] = b
        return col + b.shape[1]

    c = put(0, np.full(n, HEADER_LEN, dtype="<i4"))
    c = put(c, np.full(n, body_len, dtype="<i4"))
    c = put(c, np.full(n, MASK, dtype="<u4"))
    c = put(c, np.full(n, 2, dtype=np.uint8))                                    # Category.Application
    c = put(c, np.zeros(n, dtype=np.uint8))                                      # Direction.Request
    c = put(c, np.arange(1, n + 1, dtype="<i8"))                                 # CorrelationId
    sa = rng.integers(0, 1 << 63, size=(n, 3), dtype=np.uint64)
    sa[:, 2] = 0
    c = put(c, sa)
    c = put(c, np.full(n, -1, dtype="<i4"))
    sg = tk[rng.integers(0, n, size=n)] if sender_keys is None else np.asarray(sender_keys, dtype=np.uint64)
    c = put(c, np.ascontiguousarray(sg))
    c = put(c, np.full(n, -1, dtype="<i4"))
    silo = np.zeros((n, 24), dtype=np.uint8)
    silo[:, 12:16] = [10, 0, 0, 1]
    silo[:, 16:20] = np.frombuffer(np.int32(11111).tobytes(), dtype=np.uint8)
    silo[:, 20:24] = np.frombuffer(np.int32(138558).tobytes(), dtype=np.uint8)
    c = put(c, silo)
    c = put(c, tk)
    c = put(c, np.full(n, -1, dtype="<i4"))
    assert c == 8 + HEADER_LEN
    if body_len:
        rec[:, c:] = rng.integers(0, 256, size=(n, body_len), dtype=np.uint8)
    offsets = np.arange(n, dtype=np.uint64) * np.uint64(fl)
    return rec.reshape(-1), offsets, fl
