"""KeyExt grains -- CPU restatement (TEST INFRASTRUCTURE ONLY: the checker for the
library's KeyExt directory and routing; never imported by the product path).

String-keyed grains (IGrainWithStringKey: GrainId.GetGrainId(long typeCode, string),
GrainId.cs:86-91 -> N0 = N1 = 0), compound keys (GrainId.cs:72-84: long or Guid key +
KeyExt) and geo clients carry a KeyExt string (UniqueKey.HasKeyExt, UniqueKey.cs:60-66):
  * uniform hash = JenkinsHash.ComputeHash(ToByteArray()) when KeyExt != null
    (UniqueKey.cs:272-293), ToByteArray = N0 | N1 | TCD | int32 UTF-8 length | UTF-8
    (UniqueKey.cs:295-336, == BinaryTokenStreamWriter.Write(UniqueKey),
    Identifiertests.cs:32-48); KeyExt == null -> the three-word hash;
  * equality = the three words and the KeyExt string (UniqueKey.cs:245-251).
The library compares UTF-8 bytes.  That equals C#'s ordinal string equality except for strings
holding unpaired surrogates (Encoding.UTF8 maps each to U+FFFD, so two different strings can
share bytes): the host sends those with length EXT_HOST and they keep status KEYEXT.

Ext batches are lists whose items are bytes (UTF-8), None (KeyExt null) or EXT_HOST.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

import oracle as o

EXT_NULL = -1
EXT_HOST = "host"          # marker: the host keeps this message (status KEYEXT)


def ext_uniform_hash(n0: int, n1: int, tcd: int, ext: Optional[bytes]) -> int:
    """UniqueKey.GetUniformHashCode for a KeyExt-category key (UniqueKey.cs:272-293)."""
    if ext is None:
        return o.jenkins_u64x3(tcd, n0, n1)
    return o.jenkins_bytes(struct.pack("<QQQi", n0, n1, tcd, len(ext)) + ext)


def pack_ext(exts: Sequence) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(bytes u8[], offset u64[n], length i32[n]) in the gd_key_ext layout."""
    off = np.zeros(len(exts), np.uint64)
    ln = np.zeros(len(exts), np.int32)
    parts, pos = [], 0
    for i, e in enumerate(exts):
        if e is None:
            ln[i] = EXT_NULL
        elif isinstance(e, str) and e == EXT_HOST:
            ln[i] = -2
        else:
            off[i] = pos
            ln[i] = len(e)
            parts.append(e)
            pos += len(e)
    blob = np.frombuffer(b"".join(parts), dtype=np.uint8).copy() if parts else np.zeros(0, np.uint8)
    return blob, off, ln


class KeyExtDirectory:
    """GrainDirectoryPartition (GrainDirectoryPartition.cs:215, 304-363) restricted to KeyExt
    grains: (n0, n1, tcd, KeyExt bytes | None) -> (act, silo)."""

    def __init__(self):
        self.data: Dict[Tuple[int, int, int, Optional[bytes]], Tuple[int, int]] = {}

    @staticmethod
    def _k(key, ext):
        return (int(key[0]), int(key[1]), int(key[2]), ext)

    def add_single_activation(self, key, ext, act: int, silo: int) -> Tuple[int, int, bool]:
        """AddSingleActivation (:304-326, GrainInfo :110-124): the first registration wins."""
        k = self._k(key, ext)
        if k in self.data:
            a, s = self.data[k]
            return a, s, False
        self.data[k] = (act, silo)
        return act, silo, True

    def remove_activation(self, key, ext, act: int) -> bool:
        """RemoveActivation (:335-363): drop the entry if the activation matches."""
        k = self._k(key, ext)
        cur = self.data.get(k)
        if cur is not None and cur[0] == act:
            del self.data[k]
            return True
        return False

    def lookup(self, key, ext) -> Optional[Tuple[int, int]]:
        return self.data.get(self._k(key, ext))


def route_batch_ext(keys: np.ndarray, exts: List, spec: o.RingSpec, directory: o.DirectoryArrays,
                    kx: KeyExtDirectory, my_silo: int = 0, seed_silo: int = o.M32):
    """route_batch_np with KeyExt grains routed too: owner = CalculateTargetSilo over the KeyExt
    uniform hash (LocalGrainDirectory.cs:477-545), then the owner partition's lookup.  EXT_HOST
    items keep status KEYEXT (silo = act = none)."""
    st, silo, act, owner, h = o.route_batch_np(keys, spec, directory, my_silo=my_silo, seed_silo=seed_silo)
    keys = np.asarray(keys, dtype=np.uint64).reshape(-1, 3)
    for i in np.nonzero(st == o.ST_KEYEXT)[0]:
        e = exts[i]
        if isinstance(e, str) and e == EXT_HOST:
            continue
        n0, n1, tcd = (int(x) for x in keys[i])
        hh = ext_uniform_hash(n0, n1, tcd, e)
        own = int(o.ring_owner_np(spec, np.array([hh], np.uint32))[0])
        h[i] = hh
        owner[i] = own
        v = kx.lookup(keys[i], e)
        if v is None:
            st[i], silo[i], act[i] = o.ST_MISS, own, o.M32
        else:
            st[i] = o.ST_OK
            act[i], silo[i] = v
    return st, silo, act, owner, h


def string_grain(type_code: int, s: str) -> Tuple[Tuple[int, int, int], bytes]:
    """GrainId.GetGrainId(long typeCode, string primaryKey), GrainId.cs:86-91."""
    return (0, 0, o.type_code_data(o.CAT_KEYEXT_GRAIN, type_code)), s.encode("utf-8")
