"""ctypes binding of libgraindispatch.so (include/graindispatch.h).

This is the Python face of the C ABI that the Orleans C# host binds with
[DllImport("graindispatch")].  It holds no routing logic:
every call goes straight through the C ABI to the gfx950 kernels.  There is
no CPU fallback -- if the shared library is missing, import fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GRAINDISPATCH_LIB", os.path.join(_HERE, "libgraindispatch.so"))

# ---- constants mirrored from include/graindispatch.h --------------------------
GD_OK, GD_EINVAL, GD_ENOMEM, GD_EHIP, GD_ERCCL, GD_EFULL, GD_ESTATE, GD_ETIMEOUT = 0, -1, -2, -3, -4, -5, -6, -7
RING_DIRECTORY, RING_CONSISTENT, RING_VIRTUAL_BUCKETS = 0, 1, 2
ROUTE_OK, ROUTE_MISS, ROUTE_SYSTEM_TARGET, ROUTE_MEMBERSHIP, ROUTE_KEYEXT = 0, 1, 2, 3, 4
ROUTE_ADDRESSED, ROUTE_UNDECODED = 5, 6
FRAME_HAS_TARGET, FRAME_COMPLETE, FRAME_FALLBACK, FRAME_MALFORMED, FRAME_TARGET_KEYEXT = 1, 2, 4, 8, 16
NO_ACTIVATION = 0xFFFFFFFF
NO_SILO = 0xFFFFFFFF
CFG_KERNEL_TIMING = 1
CFG_NO_LANE_ORDER = 2

RING_MODES = {"D": RING_DIRECTORY, "R": RING_CONSISTENT, "V": RING_VIRTUAL_BUCKETS}

# C-ABI symbols the header declares (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = [
    "gd_create", "gd_destroy", "gd_last_error", "gd_abi_version", "gd_set_stream", "gd_get_stream", "gd_set_bucket_stream",
    "gd_synchronize", "gd_stats_get", "gd_host_alloc", "gd_host_free", "gd_jenkins_hash_bytes",
    "gd_jenkins_hash_u64x3", "gd_uniform_hash",
    "gd_calculate_id_hash", "gd_silo_consistent_hash", "gd_silo_uniform_hashes", "gd_silo_compare",
    "gd_ring_build", "gd_ring_set", "gd_ring_owner", "gd_ring_lookup_hashes", "gd_dir_register",
    "gd_dir_unregister", "gd_dir_lookup", "gd_dir_clear", "gd_dir_rehash", "gd_route", "gd_bucket",
    "gd_route_bucket", "gd_route_device", "gd_bucket_device", "gd_route_bucket_device",
    "gd_ring_owner_device", "gd_pack_by_shard_device", "gd_pack_routes_by_rank_device", "gd_kernel_times",
    "gd_kernel_times_reset",
    "gd_option_set", "gd_option_get", "gd_tune_reset", "gd_tune_set", "gd_tune_get", "gd_tune_agree",
    "gd_comm_info", "gd_index_stats_get", "gd_route_bound_device",
    "gd_set_kernel_timing", "gd_microbatch_create", "gd_microbatch_destroy", "gd_microbatch_keys",
    "gd_microbatch_outputs", "gd_microbatch_run", "gd_decode_frames_device", "gd_decode_frames",
    "gd_route_frames_device", "gd_route_frames", "gd_dir_split", "gd_dir_split_device",
    "gd_fanout_expand_device", "gd_fanout_route_bucket_device", "gd_fanout_route_bucket", "gd_route_nodes_device",
    "gd_pack_nodes_by_shard_device", "gd_frontier_next_device",
    "gd_cache_configure", "gd_cache_set_silos", "gd_cache_add", "gd_cache_remove", "gd_cache_lookup",
    "gd_cache_clear", "gd_cache_stats_get", "gd_cache_entries", "gd_cache_add_ext", "gd_cache_remove_ext",
    "gd_cache_lookup_ext", "gd_cache_entries_ext",
    "gd_route_frames_ext_device", "gd_route_frames_ext",
    "gd_dir_register_ext", "gd_dir_unregister_ext", "gd_dir_lookup_ext", "gd_uniform_hashes_ext",
    "gd_dir_ext_stats", "gd_route_ext", "gd_route_bucket_ext", "gd_route_ext_device", "gd_route_bucket_ext_device",
    "gd_comm_unique_id", "gd_comm_init", "gd_comm_init_local", "gd_comm_destroy", "gd_route_multi_device",
    "gd_route_multi",
    "gd_multi_fetch", "gd_route_multi_ext_device", "gd_route_multi_ext", "gd_ring_owner_ext",
    "gd_dir_split_ext", "gd_dir_upsert", "gd_dir_register_device", "gd_dir_register_device_async",
    "gd_dir_unregister_device",
    "gd_dir_set_valid_silos", "gd_dir_lookup_tagged", "gd_dir_remove_silos", "gd_activation_ids_set", "gd_dir_merge",
    "gd_actdir_add", "gd_actdir_remove", "gd_actdir_set_flags", "gd_actdir_lookup", "gd_actdir_clear",
    "gd_actdir_count", "gd_receive", "gd_receive_device", "gd_receive_frames_device", "gd_receive_frames",
    "gd_fanout_multi_device", "gd_fanout_multi", "gd_fanout_multi_fetch", "gd_dir_handoff_multi",
    "gd_fanout_multi_part_device", "gd_fanout_cascade_device",
    "gd_dir_handoff_fetch",
]


class gd_key(C.Structure):
    _fields_ = [("n0", C.c_uint64), ("n1", C.c_uint64), ("type_code_data", C.c_uint64)]


class gd_val(C.Structure):
    _fields_ = [("act", C.c_uint32), ("silo", C.c_uint32)]


class gd_silo_addr(C.Structure):
    _fields_ = [("ip", C.c_uint8 * 16), ("port", C.c_int32), ("generation", C.c_int32), ("is_v4", C.c_int32)]


class gd_config(C.Structure):
    _fields_ = [("struct_size", C.c_uint32), ("device", C.c_int32), ("table_capacity", C.c_uint64),
                ("my_silo", C.c_uint32), ("seed_silo", C.c_uint32), ("max_batch", C.c_uint32),
                ("flags", C.c_uint32)]


class gd_stats(C.Structure):
    _fields_ = [("routed", C.c_uint64), ("table_live", C.c_uint64), ("table_tombstones", C.c_uint64),
                ("table_capacity", C.c_uint64), ("ring_points", C.c_uint64), ("ring_mode", C.c_uint64)]


class gd_index_stats(C.Structure):
    _fields_ = [("builds", C.c_uint64), ("synced_slots", C.c_uint64), ("last_build_ms", C.c_double),
                ("current", C.c_uint32), ("types8", C.c_uint32), ("act_bits8", C.c_uint32),
                ("silo_bits8", C.c_uint32), ("n0_live", C.c_uint32), ("out8", C.c_uint32)]


class gd_cache_stats(C.Structure):
    _fields_ = [("count", C.c_uint64), ("accesses", C.c_uint64), ("hits", C.c_uint64),
                ("next_generation", C.c_uint64), ("max_size", C.c_uint64), ("capacity", C.c_uint64)]


class gd_kernel_time(C.Structure):
    _fields_ = [("name", C.c_char * 48), ("launches", C.c_uint64), ("total_ms", C.c_double)]


class gd_frame_fields(C.Structure):
    _fields_ = [(name, C.c_void_p) for name in
                ("flags", "target_grain", "mask", "target_activation", "sending_activation", "sending_grain",
                 "target_silo", "sending_silo", "correlation_id", "category", "direction")]


# gd_frame_fields member -> (numpy dtype, trailing shape) of the host arrays
FRAME_FIELDS = {"flags": (np.uint32, ()), "target_grain": (np.uint64, (3,)), "mask": (np.uint32, ()),
                "target_activation": (np.uint64, (3,)), "sending_activation": (np.uint64, (3,)),
                "sending_grain": (np.uint64, (3,)), "target_silo": (np.uint8, (24,)),
                "sending_silo": (np.uint8, (24,)), "correlation_id": (np.int64, ()),
                "category": (np.uint8, ()), "direction": (np.uint8, ())}


class gd_multi_result(C.Structure):
    _fields_ = [("n_recv", C.c_uint32), ("n_act", C.c_uint32)] + [
        (f, C.c_void_p) for f in ("recv_keys", "recv_idx", "recv_src", "silo", "act", "status", "perm", "offsets",
                                  "ret_silo", "ret_act", "ret_status")]


class gd_fanout_hop(C.Structure):
    _fields_ = [("n_frontier", C.c_uint32), ("frontier", C.c_void_p), ("n_sent", C.c_uint64), ("n_recv", C.c_uint32)] + [
        (f, C.c_void_p) for f in ("target", "sender", "src", "silo", "act", "status", "perm", "offsets")]


class gd_handoff_result(C.Structure):
    _fields_ = [("n_sent", C.c_uint64), ("n_recv", C.c_uint32)] + [
        (f, C.c_void_p) for f in ("recv_keys", "recv_ids", "recv_act", "recv_silo", "recv_src", "status", "dropped")]


GD_HANDOFF_ADD, GD_HANDOFF_REMOVE = 0, 1
GD_MERGE_TAG_MULTI_INSTANCE = 0x80000000
GD_MERGE_INSERTED, GD_MERGE_KEPT, GD_MERGE_SAME, GD_MERGE_DROPPED, GD_MERGE_HOST, GD_MERGE_UNION = 0, 1, 2, 3, 4, 5
ACTDIR_VALID, ACTDIR_SYSTEM_TARGET, ACTDIR_STATELESS_WORKER = 1, 2, 4
(RECV_ACTIVATION, RECV_SYSTEM_TARGET, RECV_NULL_CONTEXT, RECV_REJECT_UNKNOWN, RECV_REJECT_OVERLOADED, RECV_DROPPED,
 RECV_UNDECODED) = range(7)


class gd_recv_limits(C.Structure):
    _fields_ = [("request_count", C.c_void_p), ("hard_limit", C.c_int32), ("hard_limit_stateless_worker", C.c_int32)]


GD_COMM_ID_BYTES = 128
GD_ACT_MULTI = 0xFFFFFFFE
GD_ROUTE_MULTI_ACT = 7
GD_KEYEXT_NULL = -1
GD_KEYEXT_HOST = -2


class gd_key_ext(C.Structure):
    _fields_ = [("bytes", C.c_void_p), ("offset", C.c_void_p), ("length", C.c_void_p), ("bytes_len", C.c_uint64)]


class KeyExtBatch:
    """A batch's KeyExt strings in the gd_key_ext layout.  Items: bytes (UTF-8), str (encoded
    UTF-8), None (KeyExt null) or GD_KEYEXT_HOST (leave to the C# path).  Holds the arrays the
    struct points at."""

    def __init__(self, exts):
        n = len(exts)
        self.offset = np.zeros(n, np.uint64)
        self.length = np.zeros(n, np.int32)
        parts, pos = [], 0
        for i, e in enumerate(exts):
            if e is None:
                self.length[i] = GD_KEYEXT_NULL
            elif isinstance(e, (int, np.integer)):
                self.length[i] = int(e)
            else:
                b = e.encode("utf-8") if isinstance(e, str) else bytes(e)
                self.offset[i] = pos
                self.length[i] = len(b)
                parts.append(b)
                pos += len(b)
        self.blob = np.frombuffer(b"".join(parts) + b"\0", dtype=np.uint8).copy()
        self.struct = gd_key_ext(self.blob.ctypes.data, self.offset.ctypes.data, self.length.ctypes.data, pos)


GD_MULTI_RETURN_ROUTES = 1
GD_MULTI_KEYS_READY = 2
GD_MULTI_FORWARD = 4
GD_MULTI_NO_KEYS = 8


class GrainDispatchError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"graindispatch error {code}: {msg}")
        self.code = code


def _load() -> C.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libgraindispatch.so not built at {LIB_PATH}; run __graft_entry__.build()")
    # One HIP runtime per process.  torch ships its own libamdhip64 / libhsa-runtime64 with the
    # same sonames as /opt/rocm's but is linked against the unversioned names: if this library
    # loaded /opt/rocm's copies first, a later `import torch` would load its copies beside them
    # and whichever HSA runtime initialises second finds no device.  With torch imported first,
    # our NEEDED libamdhip64.so.7 resolves to the copy torch already holds.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(LIB_PATH)
    P, U32, U64, I32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int32
    sig = {
        "gd_create": (C.c_int, [C.POINTER(gd_config), C.POINTER(P)]),
        "gd_destroy": (None, [P]),
        "gd_last_error": (C.c_char_p, [P]),
        "gd_abi_version": (C.c_int, []),
        "gd_set_stream": (C.c_int, [P, P]),
        "gd_set_bucket_stream": (C.c_int, [P, P]),
        "gd_get_stream": (P, [P]),
        "gd_host_alloc": (C.c_int, [C.c_size_t, P]),
        "gd_host_free": (C.c_int, [P]),
        "gd_synchronize": (C.c_int, [P]),
        "gd_stats_get": (C.c_int, [P, C.POINTER(gd_stats)]),
        "gd_index_stats_get": (C.c_int, [P, C.POINTER(gd_index_stats)]),
        "gd_jenkins_hash_bytes": (U32, [P, C.c_size_t]),
        "gd_jenkins_hash_u64x3": (U32, [U64, U64, U64]),
        "gd_uniform_hash": (U32, [C.POINTER(gd_key)]),
        "gd_calculate_id_hash": (I32, [C.c_char_p]),
        "gd_silo_consistent_hash": (I32, [C.POINTER(gd_silo_addr)]),
        "gd_silo_uniform_hashes": (C.c_int, [C.POINTER(gd_silo_addr), U32, P]),
        "gd_silo_compare": (C.c_int, [C.POINTER(gd_silo_addr), C.POINTER(gd_silo_addr)]),
        "gd_ring_build": (C.c_int, [C.c_int, P, U32, U32, P, P, C.POINTER(U32)]),
        "gd_ring_set": (C.c_int, [P, C.c_int, P, P, U32]),
        "gd_ring_owner": (C.c_int, [P, P, U32, P]),
        "gd_ring_lookup_hashes": (C.c_int, [P, P, U32, P]),
        "gd_dir_register": (C.c_int, [P, P, P, U32, P, P]),
        "gd_dir_unregister": (C.c_int, [P, P, P, U32, P]),
        "gd_dir_register_device": (C.c_int, [P, P, P, U32, P, P]),
        "gd_dir_register_device_async": (C.c_int, [P, P, P, U32, P, P]),
        "gd_dir_unregister_device": (C.c_int, [P, P, P, U32, P]),
        "gd_dir_set_valid_silos": (C.c_int, [P, P, U32]),
        "gd_dir_lookup_tagged": (C.c_int, [P, P, U32, P, P, P]),
        "gd_dir_remove_silos": (C.c_int, [P, P, U32, C.POINTER(U64), C.POINTER(U64), C.POINTER(U64)]),
        "gd_activation_ids_set": (C.c_int, [P, P, P, U32]),
        "gd_dir_merge": (C.c_int, [P, P, P, P, U32, P, P]),
        "gd_actdir_add": (C.c_int, [P, P, P, P, U32, P]),
        "gd_actdir_remove": (C.c_int, [P, P, U32, P]),
        "gd_actdir_set_flags": (C.c_int, [P, P, P, U32, P]),
        "gd_actdir_lookup": (C.c_int, [P, P, U32, P, P, P]),
        "gd_actdir_clear": (C.c_int, [P]),
        "gd_actdir_count": (C.c_int, [P, C.POINTER(U64)]),
        "gd_receive": (C.c_int, [P, P, P, P, U32, U32, C.POINTER(gd_recv_limits), P, P, P, P]),
        "gd_receive_device": (C.c_int, [P, P, P, P, U32, U32, C.POINTER(gd_recv_limits), P, P, P, P]),
        "gd_receive_frames_device": (C.c_int, [P, P, U64, P, U32, U32, C.POINTER(gd_recv_limits),
                                               C.POINTER(gd_frame_fields), P, P, P, P]),
        "gd_receive_frames": (C.c_int, [P, P, U64, P, U32, U32, C.POINTER(gd_recv_limits), C.POINTER(gd_frame_fields),
                                        P, P, P, P]),
        "gd_dir_upsert": (C.c_int, [P, P, P, U32, P]),
        "gd_dir_lookup": (C.c_int, [P, P, U32, P, P]),
        "gd_dir_clear": (C.c_int, [P]),
        "gd_dir_rehash": (C.c_int, [P, U64]),
        "gd_route": (C.c_int, [P, P, U32, P, P, P]),
        "gd_bucket": (C.c_int, [P, P, U32, U32, P, P]),
        "gd_route_bucket": (C.c_int, [P, P, U32, U32, P, P, P, P, P]),
        "gd_route_device": (C.c_int, [P, P, U32, P, P, P]),
        "gd_route_bound_device": (C.c_int, [P, P, U32, P, P, P]),
        "gd_bucket_device": (C.c_int, [P, P, U32, U32, P, P]),
        "gd_route_bucket_device": (C.c_int, [P, P, U32, U32, P, P, P, P, P]),
        "gd_ring_owner_device": (C.c_int, [P, P, U32, P]),
        "gd_pack_by_shard_device": (C.c_int, [P, P, U32, U32, P, P, P]),
        "gd_pack_routes_by_rank_device": (C.c_int, [P, P, P, P, U32, U32, U32, P, P, P]),
        "gd_kernel_times": (C.c_int, [P, C.POINTER(gd_kernel_time), U32, C.POINTER(U32)]),
        "gd_kernel_times_reset": (C.c_int, [P]),
        "gd_set_kernel_timing": (C.c_int, [P, C.c_int]),
        "gd_microbatch_create": (C.c_int, [P, U32, U32, C.POINTER(P)]),
        "gd_microbatch_destroy": (None, [P]),
        "gd_microbatch_keys": (P, [P]),
        "gd_microbatch_outputs": (C.c_int, [P] + [C.POINTER(P)] * 7),
        "gd_microbatch_run": (C.c_int, [P, U32, C.c_int]),
        "gd_decode_frames_device": (C.c_int, [P, P, U64, P, U32, C.POINTER(gd_frame_fields)]),
        "gd_decode_frames": (C.c_int, [P, P, U64, P, U32, C.POINTER(gd_frame_fields)]),
        "gd_route_frames_device": (C.c_int, [P, P, U64, P, U32, U32, C.POINTER(gd_frame_fields), P, P, P, P, P]),
        "gd_route_frames": (C.c_int, [P, P, U64, P, U32, U32, C.POINTER(gd_frame_fields), P, P, P, P, P]),
        "gd_route_frames_ext_device": (C.c_int, [P, P, U64, P, U32, U32, C.POINTER(gd_frame_fields), P, P, P, P, P]),
        "gd_route_frames_ext": (C.c_int, [P, P, U64, P, U32, U32, C.POINTER(gd_frame_fields), P, P, P, P, P]),
        "gd_dir_split": (C.c_int, [P, P, U32, C.c_int, P, P, U64, C.POINTER(U64)]),
        "gd_dir_split_device": (C.c_int, [P, P, U32, C.c_int, P, P, U64, C.POINTER(U64)]),
        "gd_fanout_expand_device": (C.c_int, [P, P, P, U32, P, U32, P, P, U64, C.POINTER(U64)]),
        "gd_fanout_route_bucket_device": (C.c_int, [P, P, P, U32, P, U32, I32, U32] + [P] * 7 + [U64, C.POINTER(U64)]),
        "gd_fanout_route_bucket": (C.c_int, [P, P, P, U32, P, U32, I32, U32] + [P] * 7 + [U64, C.POINTER(U64)]),
        "gd_route_nodes_device": (C.c_int, [P, P, U32, I32, P, P, P]),
        "gd_pack_nodes_by_shard_device": (C.c_int, [P, P, P, U32, I32, U32, P, P, P]),
        "gd_frontier_next_device": (C.c_int, [P, P, U32, P, P, C.POINTER(U32)]),
        "gd_cache_configure": (C.c_int, [P, U32, P, P, U32]),
        "gd_cache_set_silos": (C.c_int, [P, P, P, U32]),
        "gd_cache_add": (C.c_int, [P, P, P, P, U32]),
        "gd_cache_remove": (C.c_int, [P, P, U32, P]),
        "gd_cache_lookup": (C.c_int, [P, P, U32, P, P, P]),
        "gd_cache_clear": (C.c_int, [P]),
        "gd_cache_stats_get": (C.c_int, [P, C.POINTER(gd_cache_stats)]),
        "gd_cache_entries": (C.c_int, [P, P, P, P, P, U64, C.POINTER(U64)]),
        "gd_cache_add_ext": (C.c_int, [P, P, C.POINTER(gd_key_ext), P, P, U32]),
        "gd_cache_remove_ext": (C.c_int, [P, P, C.POINTER(gd_key_ext), U32, P]),
        "gd_cache_lookup_ext": (C.c_int, [P, P, C.POINTER(gd_key_ext), U32, P, P, P]),
        "gd_cache_entries_ext": (C.c_int, [P, P, P, P, P, P, P, P, U64, U64, C.POINTER(U64), C.POINTER(U64)]),
        "gd_dir_register_ext": (C.c_int, [P, P, C.POINTER(gd_key_ext), P, U32, P, P]),
        "gd_dir_unregister_ext": (C.c_int, [P, P, C.POINTER(gd_key_ext), P, U32, P]),
        "gd_dir_lookup_ext": (C.c_int, [P, P, C.POINTER(gd_key_ext), U32, P, P]),
        "gd_uniform_hashes_ext": (C.c_int, [P, P, C.POINTER(gd_key_ext), U32, P]),
        "gd_dir_ext_stats": (C.c_int, [P, C.POINTER(U64), C.POINTER(U64), C.POINTER(U64)]),
        "gd_route_ext": (C.c_int, [P, P, C.POINTER(gd_key_ext), U32, P, P, P]),
        "gd_route_bucket_ext": (C.c_int, [P, P, C.POINTER(gd_key_ext), U32, U32, P, P, P, P, P]),
        "gd_route_ext_device": (C.c_int, [P, P, C.POINTER(gd_key_ext), U32, P, P, P]),
        "gd_route_bucket_ext_device": (C.c_int, [P, P, C.POINTER(gd_key_ext), U32, U32, P, P, P, P, P]),
        "gd_comm_unique_id": (C.c_int, [P]),
        "gd_comm_init": (C.c_int, [P, P, C.c_int, C.c_int]),
        "gd_comm_init_local": (C.c_int, [P, C.c_int]),
        "gd_comm_destroy": (C.c_int, [P]),
        "gd_route_multi_device": (C.c_int, [P, P, U32, U32, C.c_int, C.POINTER(gd_multi_result)]),
        "gd_route_multi": (C.c_int, [P, P, U32, U32, C.c_int, C.POINTER(gd_multi_result)]),
        "gd_multi_fetch": (C.c_int, [P] + [P] * 11),
        "gd_route_multi_ext_device": (C.c_int, [P, P, C.POINTER(gd_key_ext), U32, U32, C.c_int,
                                                C.POINTER(gd_multi_result)]),
        "gd_ring_owner_ext": (C.c_int, [P, P, C.POINTER(gd_key_ext), U32, P]),
        "gd_dir_split_ext": (C.c_int, [P, P, U32, C.c_int, P, P, P, P, P, U64, U64, C.POINTER(U64), C.POINTER(U64)]),
        "gd_route_multi_ext": (C.c_int, [P, P, C.POINTER(gd_key_ext), U32, U32, C.c_int, C.POINTER(gd_multi_result)]),
        "gd_fanout_multi_device": (C.c_int, [P, P, P, U32, P, U32, C.c_int32, U32, U32, P]),
        "gd_fanout_multi_part_device": (C.c_int, [P, P, P, U32, P, P, U32, C.c_int32, U32, P]),
        "gd_fanout_cascade_device": (C.c_int, [P, P, P, U32, P, U32, C.c_int32, U32, U32, P]),
        "gd_fanout_multi": (C.c_int, [P, P, P, U32, P, U32, C.c_int32, U32, U32, P]),
        "gd_fanout_multi_fetch": (C.c_int, [P, U32] + [P] * 9),
        "gd_dir_handoff_multi": (C.c_int, [P, P, U32, C.c_int, U32, C.POINTER(gd_handoff_result)]),
        "gd_dir_handoff_fetch": (C.c_int, [P] + [P] * 7),
        "gd_option_set": (C.c_int, [P, C.c_int, C.c_int64]),
        "gd_option_get": (C.c_int, [P, C.c_int, C.POINTER(C.c_int64)]),
        "gd_tune_reset": (C.c_int, [P]),
        "gd_tune_set": (C.c_int, [P, C.c_int, C.c_int]),
        "gd_tune_get": (C.c_int, [P, C.c_int, U64, U32, C.POINTER(C.c_int)]),
        "gd_tune_agree": (C.c_int, [P]),
        "gd_comm_info": (C.c_int, [P, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    }
    ab_variant = "GRAINDISPATCH_LIB" in os.environ     # an older build for an A/B: its missing entry points stay unbound
    for name, (res, args) in sig.items():
        fn = getattr(lib, name, None)
        if fn is None and ab_variant:
            continue
        if fn is None:
            raise ImportError(f"{LIB_PATH} lacks {name}: rebuild it (__graft_entry__.build())")
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def keys_array(keys) -> np.ndarray:
    """(N,3) uint64 [n0, n1, type_code_data] in C order (the gd_key AoS layout)."""
    k = np.ascontiguousarray(np.asarray(keys, dtype=np.uint64).reshape(-1, 3))
    return k


# ---- identity helpers ------------------------------------------------------------

def silo_addr(ip: str, port: int, gen: int) -> gd_silo_addr:
    import ipaddress
    a = ipaddress.ip_address(ip)
    s = gd_silo_addr()
    raw = (b"\x00" * 12 + a.packed) if a.version == 4 else a.packed
    for i, b in enumerate(raw):
        s.ip[i] = b
    s.port, s.generation, s.is_v4 = port, gen, 1 if a.version == 4 else 0
    return s


def jenkins_bytes(data: bytes) -> int:
    buf = (C.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    return lib.gd_jenkins_hash_bytes(buf, len(data))


def jenkins_u64x3(u1: int, u2: int, u3: int) -> int:
    return lib.gd_jenkins_hash_u64x3(u1, u2, u3)


def calculate_id_hash(text: str) -> int:
    return lib.gd_calculate_id_hash(text.encode("utf-8"))


def silo_consistent_hash(ip: str, port: int, gen: int) -> int:
    return lib.gd_silo_consistent_hash(C.byref(silo_addr(ip, port, gen)))


def silo_uniform_hashes(ip: str, port: int, gen: int, n: int) -> List[int]:
    out = np.zeros(max(n, 1), dtype=np.uint32)
    _check(None, lib.gd_silo_uniform_hashes(C.byref(silo_addr(ip, port, gen)), n, _ptr(out)))
    return [int(x) for x in out[:n]]


def ring_build(mode: str, silos: Sequence[Tuple[str, int, int]], buckets: int = 30) -> Tuple[np.ndarray, np.ndarray]:
    """LocalGrainDirectory / ConsistentRingProvider / VirtualBucketsRingProvider
    AddServer over `silos` (added in order).  Returns (points u32, owner u32)."""
    m = RING_MODES[mode] if isinstance(mode, str) else mode
    arr = (gd_silo_addr * len(silos))(*[silo_addr(*s) for s in silos])
    cap = len(silos) * (buckets if m == RING_VIRTUAL_BUCKETS else 1)
    pts = np.zeros(cap, dtype=np.uint32)
    own = np.zeros(cap, dtype=np.uint32)
    n = C.c_uint32(0)
    _check(None, lib.gd_ring_build(m, arr, len(silos), buckets, _ptr(pts), _ptr(own), C.byref(n)))
    return pts[: n.value].copy(), own[: n.value].copy()


def _check(h, rc: int):
    if rc != GD_OK:
        msg = lib.gd_last_error(h)
        raise GrainDispatchError(rc, msg.decode() if msg else "")


# ---- handle options (include/graindispatch.h GD_OPT_*) and measured choices (GD_TUNE_*) -----------
OPTIONS = {"probe": 1, "bucket": 2, "l2_small": 3, "stable_rank": 4, "wire_headers": 5, "region_probe": 6,
           "idx16": 7, "host_chunk": 8, "mb_zerocopy": 9, "mb_split": 10, "mb_trace": 11, "l2_staged": 12,
           "l2_mid": 13, "b2_persist": 14, "b2_order": 15, "mb_poll": 16,
           "fan_bound": 17}
TUNE_KINDS = {"probe_keys": 0, "probe_n1": 1, "probe_fanout": 2, "probe_nodes": 3, "bucket": 4}
# Options applied to every handle this process creates, before its own `options=` (the test and tool
# harness sets these; a C# host calls gd_option_set on its handle instead).
DEFAULT_OPTIONS: dict = {}
# Every handle created as if its device failed gd_create's lane-order check (GD_CFG_NO_LANE_ORDER): the
# test suite's ballot-rank run (tests/conftest.py, GD_TEST_BALLOT_RANKS=1) sets it
FORCE_NO_LANE_ORDER = False


# ---- the handle --------------------------------------------------------------------

class GrainDispatch:
    """One libgraindispatch handle: a ring snapshot + the directory partitions this
    GPU owns + scratch, on one HIP stream."""

    def __init__(self, device: int = 0, table_capacity: int = 1 << 20, my_silo: int = 0,
                 seed_silo: int = NO_SILO, kernel_timing: bool = False, options: Optional[dict] = None,
                 no_lane_order: bool = False):
        """no_lane_order (GD_CFG_NO_LANE_ORDER): the handle behaves as on a device that fails gd_create's
        LDS lane-order check -- every stable rank by ballots."""
        cfg = gd_config(C.sizeof(gd_config), device, table_capacity, my_silo, seed_silo, 0,
                        (CFG_KERNEL_TIMING if kernel_timing else 0) |
                        (CFG_NO_LANE_ORDER if no_lane_order or FORCE_NO_LANE_ORDER else 0))
        h = C.c_void_p()
        _check(None, lib.gd_create(C.byref(cfg), C.byref(h)))
        self.h = h
        self.device = device
        for k, v in {**DEFAULT_OPTIONS, **(options or {})}.items():
            self.set_option(k, v)

    # -- options and measured choices ------------------------------------------
    def set_option(self, name, value: int):
        self._c(lib.gd_option_set(self.h, OPTIONS[name] if isinstance(name, str) else name, int(value)))

    def get_option(self, name) -> int:
        v = C.c_int64(0)
        self._c(lib.gd_option_get(self.h, OPTIONS[name] if isinstance(name, str) else name, C.byref(v)))
        return v.value

    def tune_reset(self):
        self._c(lib.gd_tune_reset(self.h))

    def tune_set(self, kind, variant: int):
        self._c(lib.gd_tune_set(self.h, TUNE_KINDS[kind] if isinstance(kind, str) else kind, variant))

    def tune_get(self, kind, n: int, sub: int = 0) -> int:
        v = C.c_int(0)
        self._c(lib.gd_tune_get(self.h, TUNE_KINDS[kind] if isinstance(kind, str) else kind, n, sub, C.byref(v)))
        return v.value

    def tune_agree(self):
        """Collective over the handle's communicator: every rank keeps the same measured choices."""
        self._c(lib.gd_tune_agree(self.h))

    def comm_info(self) -> dict:
        """{"n_ranks", "rank", "transport"} of the handle's communicator (RCCL's own count)."""
        nr, rk, tr = C.c_int(0), C.c_int(0), C.c_int(0)
        self._c(lib.gd_comm_info(self.h, C.byref(nr), C.byref(rk), C.byref(tr)))
        return {"n_ranks": nr.value, "rank": rk.value,
                "transport": {0: "none", 1: "rccl", 2: "in-process"}.get(tr.value, str(tr.value))}

    def close(self):
        if getattr(self, "h", None):
            lib.gd_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _c(self, rc):
        _check(self.h, rc)

    # -- stream ---------------------------------------------------------------
    def set_stream(self, hip_stream: Optional[int]):
        self._c(lib.gd_set_stream(self.h, C.c_void_p(hip_stream or 0)))

    def set_bucket_stream(self, hip_stream: Optional[int]):
        """gd_set_bucket_stream: route_bucket_device's bucketing on this stream, after the route."""
        self._c(lib.gd_set_bucket_stream(self.h, C.c_void_p(hip_stream or 0)))

    def synchronize(self):
        self._c(lib.gd_synchronize(self.h))

    def stats(self) -> dict:
        s = gd_stats()
        self._c(lib.gd_stats_get(self.h, C.byref(s)))
        return {f: getattr(s, f) for f, _ in gd_stats._fields_}

    def index_stats(self) -> dict:
        """gd_index_stats_get: builds, slots re-projected by directory batches, the 8-B layout."""
        s = gd_index_stats()
        self._c(lib.gd_index_stats_get(self.h, C.byref(s)))
        return {f: getattr(s, f) for f, _ in gd_index_stats._fields_}

    # -- ring -----------------------------------------------------------------
    def ring_set(self, mode, points, owner):
        m = RING_MODES[mode] if isinstance(mode, str) else mode
        p = np.ascontiguousarray(np.asarray(points, dtype=np.int64).astype(np.uint32) if np.asarray(points).dtype.kind == "i"
                                 else np.asarray(points, dtype=np.uint32))
        o = np.ascontiguousarray(np.asarray(owner, dtype=np.uint32))
        self._c(lib.gd_ring_set(self.h, m, _ptr(p), _ptr(o), len(p)))

    def ring_set_silos(self, mode: str, silos, buckets: int = 30):
        pts, own = ring_build(mode, silos, buckets)
        self.ring_set(mode, pts, own)
        return pts, own

    def ring_owner(self, keys) -> np.ndarray:
        k = keys_array(keys)
        out = np.zeros(len(k), dtype=np.uint32)
        self._c(lib.gd_ring_owner(self.h, _ptr(k), len(k), _ptr(out)))
        return out

    def ring_lookup_hashes(self, hashes) -> np.ndarray:
        hs = np.ascontiguousarray(np.asarray(hashes, dtype=np.uint32))
        out = np.zeros(len(hs), dtype=np.uint32)
        self._c(lib.gd_ring_lookup_hashes(self.h, _ptr(hs), len(hs), _ptr(out)))
        return out

    # -- directory ------------------------------------------------------------
    def register(self, keys, acts, silos):
        k = keys_array(keys)
        n = len(k)
        vals = np.zeros((n, 2), dtype=np.uint32)
        vals[:, 0] = acts
        vals[:, 1] = silos
        out = np.zeros((n, 2), dtype=np.uint32)
        ins = np.zeros(n, dtype=np.uint8)
        self._c(lib.gd_dir_register(self.h, _ptr(k), _ptr(vals), n, _ptr(out), _ptr(ins)))
        return out[:, 0].copy(), out[:, 1].copy(), ins

    def register_device(self, d_keys: int, d_vals: int, n: int, d_out_vals: Optional[int] = None,
                        d_out_inserted: Optional[int] = None):
        """gd_dir_register_device: keys (n,3) u64 and values (n,2) u32 [act, silo] in HBM."""
        self._c(lib.gd_dir_register_device(self.h, C.c_void_p(d_keys), C.c_void_p(d_vals), n,
                                           C.c_void_p(d_out_vals or 0), C.c_void_p(d_out_inserted or 0)))

    def register_device_async(self, d_keys: int, d_vals: int, n: int, d_out_vals: Optional[int] = None,
                              d_out_inserted: Optional[int] = None):
        """gd_dir_register_device_async: enqueued only (device errors at the next synchronising call)."""
        self._c(lib.gd_dir_register_device_async(self.h, C.c_void_p(d_keys), C.c_void_p(d_vals), n,
                                                 C.c_void_p(d_out_vals or 0), C.c_void_p(d_out_inserted or 0)))

    def unregister_device(self, d_keys: int, d_acts: int, n: int, d_out_removed: Optional[int] = None):
        """gd_dir_unregister_device: RemoveActivation over device arrays, enqueued only."""
        self._c(lib.gd_dir_unregister_device(self.h, C.c_void_p(d_keys), C.c_void_p(d_acts), n,
                                             C.c_void_p(d_out_removed or 0)))

    # -- membership change: IsValidSilo, VersionTag, silo removal, merge ----------
    def set_valid_silos(self, valid_silos, n_silos: int):
        """gd_dir_set_valid_silos: the silos of [0, n_silos) that are valid (IsValidSilo); n_silos 0 =
        every silo valid."""
        m = np.zeros(max(n_silos, 1), dtype=np.uint8)
        if n_silos:
            m[[int(x) for x in valid_silos]] = 1
        self._c(lib.gd_dir_set_valid_silos(self.h, _ptr(m), n_silos))

    def lookup_tagged(self, keys):
        """LookUpActivations with VersionTag: (act, silo, tag i32, found u8: 0 absent, 1 valid, 2 invalid silo)."""
        k = keys_array(keys)
        n = len(k)
        vals = np.zeros((n, 2), np.uint32)
        tags = np.zeros(n, np.int32)
        found = np.zeros(n, np.uint8)
        self._c(lib.gd_dir_lookup_tagged(self.h, _ptr(k), n, _ptr(vals), _ptr(tags), _ptr(found)))
        return vals[:, 0].copy(), vals[:, 1].copy(), tags, found

    def remove_silos(self, silos) -> dict:
        """AdjustLocalDirectory (+ AdjustLocalCache in LocalLookup mode) for removed silos."""
        a = np.ascontiguousarray(np.asarray(list(silos), dtype=np.uint32))
        r, m, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self._c(lib.gd_dir_remove_silos(self.h, _ptr(a) if len(a) else None, len(a), C.byref(r), C.byref(m),
                                        C.byref(c)))
        return {"removed": r.value, "multi": m.value, "cache_removed": c.value}

    def activation_ids_set(self, acts, ids):
        a = np.ascontiguousarray(np.asarray(acts, dtype=np.uint32))
        k = keys_array(ids)
        self._c(lib.gd_activation_ids_set(self.h, _ptr(a), _ptr(k), len(a)))

    def merge(self, keys, acts, silos, tags=None):
        """gd_dir_merge: (status u8, dropped act u32, dropped silo u32)."""
        k = keys_array(keys)
        n = len(k)
        vals = np.zeros((n, 2), np.uint32)
        vals[:, 0] = acts
        vals[:, 1] = silos
        t = None if tags is None else np.ascontiguousarray(np.asarray(tags, dtype=np.int32))
        st = np.zeros(n, np.uint8)
        dr = np.zeros((n, 2), np.uint32)
        self._c(lib.gd_dir_merge(self.h, _ptr(k), _ptr(vals), None if t is None else _ptr(t), n, _ptr(st), _ptr(dr)))
        return st, dr[:, 0].copy(), dr[:, 1].copy()

    # -- receive path: ActivationDirectory + IncomingMessageAgent ------------------
    def actdir_add(self, ids, ctx, flags) -> np.ndarray:
        k = keys_array(ids)
        c = np.ascontiguousarray(np.asarray(ctx, dtype=np.uint32))
        f = np.ascontiguousarray(np.asarray(flags, dtype=np.uint8))
        out = np.zeros(len(k), np.uint8)
        self._c(lib.gd_actdir_add(self.h, _ptr(k), _ptr(c), _ptr(f), len(k), _ptr(out)))
        return out

    def actdir_remove(self, ids) -> np.ndarray:
        k = keys_array(ids)
        out = np.zeros(len(k), np.uint8)
        self._c(lib.gd_actdir_remove(self.h, _ptr(k), len(k), _ptr(out)))
        return out

    def actdir_set_flags(self, ids, flags) -> np.ndarray:
        k = keys_array(ids)
        f = np.ascontiguousarray(np.asarray(flags, dtype=np.uint8))
        out = np.zeros(len(k), np.uint8)
        self._c(lib.gd_actdir_set_flags(self.h, _ptr(k), _ptr(f), len(k), _ptr(out)))
        return out

    def actdir_lookup(self, ids):
        k = keys_array(ids)
        n = len(k)
        c = np.zeros(n, np.uint32)
        f = np.zeros(n, np.uint8)
        found = np.zeros(n, np.uint8)
        self._c(lib.gd_actdir_lookup(self.h, _ptr(k), n, _ptr(c), _ptr(f), _ptr(found)))
        return c, f, found

    def actdir_clear(self):
        self._c(lib.gd_actdir_clear(self.h))

    def actdir_count(self) -> int:
        v = C.c_uint64()
        self._c(lib.gd_actdir_count(self.h, C.byref(v)))
        return v.value

    @staticmethod
    def _limits(request_count, hard_limit, hard_limit_sw):
        if request_count is None:
            return None, None
        rc = np.ascontiguousarray(np.asarray(request_count, dtype=np.uint32))
        return gd_recv_limits(_ptr(rc), hard_limit, hard_limit_sw), rc

    def receive(self, target_grain, target_activation, direction, n_ctx: int, request_count=None, hard_limit: int = 0,
                hard_limit_sw: int = 0, bucket: bool = True):
        """gd_receive: (ctx u32, status u8[, perm, offsets[n_ctx + 3]])."""
        tg = keys_array(target_grain)
        ta = keys_array(target_activation)
        n = len(tg)
        d = None if direction is None else np.ascontiguousarray(np.asarray(direction, dtype=np.uint8))
        lim, keep = self._limits(request_count, hard_limit, hard_limit_sw)
        ctx = np.zeros(n, np.uint32)
        st = np.zeros(n, np.uint8)
        perm = np.zeros(n, np.uint32) if bucket else None
        off = np.zeros(n_ctx + 3, np.uint32) if bucket else None
        self._c(lib.gd_receive(self.h, _ptr(tg), _ptr(ta), None if d is None else _ptr(d), n, n_ctx,
                               None if lim is None else C.byref(lim), _ptr(ctx), _ptr(st),
                               None if perm is None else _ptr(perm), None if off is None else _ptr(off)))
        return (ctx, st, perm, off) if bucket else (ctx, st)

    def receive_frames(self, buf: bytes, offsets, n_ctx: int, request_count=None, hard_limit: int = 0,
                       hard_limit_sw: int = 0, fields: Optional[Iterable[str]] = ()):
        """gd_receive_frames: (decoded fields, ctx, status, perm, offsets)."""
        b = np.frombuffer(buf, dtype=np.uint8) if len(buf) else np.zeros(1, dtype=np.uint8)
        off = np.ascontiguousarray(np.asarray(offsets, dtype=np.uint64))
        n = len(off)
        arrs, ff = self._frame_host(n, fields)
        lim, keep = self._limits(request_count, hard_limit, hard_limit_sw)
        ctx = np.zeros(n, np.uint32)
        st = np.zeros(n, np.uint8)
        perm = np.zeros(n, np.uint32)
        offs = np.zeros(n_ctx + 3, np.uint32)
        self._c(lib.gd_receive_frames(self.h, _ptr(b), len(buf), _ptr(off), n, n_ctx,
                                      None if lim is None else C.byref(lim), C.byref(ff), _ptr(ctx), _ptr(st),
                                      _ptr(perm), _ptr(offs)))
        return arrs, ctx, st, perm, offs

    def receive_device(self, d_tg: int, d_ta: int, d_dir: Optional[int], n: int, n_ctx: int, d_ctx: int, d_status: int,
                       d_perm: Optional[int], d_offsets: Optional[int], d_request_count: Optional[int] = None,
                       hard_limit: int = 0, hard_limit_sw: int = 0):
        lim = gd_recv_limits(d_request_count, hard_limit, hard_limit_sw) if d_request_count else None
        self._c(lib.gd_receive_device(self.h, C.c_void_p(d_tg), C.c_void_p(d_ta), C.c_void_p(d_dir or 0), n, n_ctx,
                                      None if lim is None else C.byref(lim), C.c_void_p(d_ctx), C.c_void_p(d_status),
                                      C.c_void_p(d_perm or 0), C.c_void_p(d_offsets or 0)))

    def upsert(self, keys, acts, silos) -> np.ndarray:
        """gd_dir_upsert: overwrite, the last item of a grain wins; acts may hold GD_ACT_MULTI."""
        k = keys_array(keys)
        n = len(k)
        vals = np.zeros((n, 2), dtype=np.uint32)
        vals[:, 0] = acts
        vals[:, 1] = silos
        ins = np.zeros(n, dtype=np.uint8)
        self._c(lib.gd_dir_upsert(self.h, _ptr(k), _ptr(vals), n, _ptr(ins)))
        return ins

    def unregister(self, keys, acts) -> np.ndarray:
        k = keys_array(keys)
        a = np.ascontiguousarray(np.asarray(acts, dtype=np.uint32))
        out = np.zeros(len(k), dtype=np.uint8)
        self._c(lib.gd_dir_unregister(self.h, _ptr(k), _ptr(a), len(k), _ptr(out)))
        return out

    def lookup(self, keys):
        k = keys_array(keys)
        n = len(k)
        out = np.zeros((n, 2), dtype=np.uint32)
        found = np.zeros(n, dtype=np.uint8)
        self._c(lib.gd_dir_lookup(self.h, _ptr(k), n, _ptr(out), _ptr(found)))
        return out[:, 0].copy(), out[:, 1].copy(), found

    def clear(self):
        self._c(lib.gd_dir_clear(self.h))

    def split(self, keep_silos, move: bool = True):
        """GrainDirectoryPartition.Split by "owner under the installed ring is not kept here"
        (SURVEY 8 f4).  keep_silos: iterable of silo indices this handle keeps.  Returns
        (keys (n,3) u64, acts u32, silos u32) in slot order; move=True removes them here."""
        ks = [int(x) for x in keep_silos]
        keep = np.zeros(max(ks) + 1 if ks else 1, dtype=np.uint8)
        keep[ks] = 1
        n = C.c_uint64(0)
        self._c(lib.gd_dir_split(self.h, _ptr(keep), len(keep), 1 if move else 0, None, None, 0, C.byref(n)))
        keys = np.zeros((n.value, 3), dtype=np.uint64)
        vals = np.zeros((n.value, 2), dtype=np.uint32)
        if n.value:
            got = C.c_uint64(0)
            self._c(lib.gd_dir_split(self.h, _ptr(keep), len(keep), 1 if move else 0, _ptr(keys), _ptr(vals),
                                     n.value, C.byref(got)))
            assert got.value == n.value
        return keys, vals[:, 0].copy(), vals[:, 1].copy()

    @staticmethod
    def keep_mask(keep_silos, n_silos: int) -> np.ndarray:
        keep = np.zeros(max(n_silos, 1), dtype=np.uint8)
        keep[[int(x) for x in keep_silos]] = 1
        return keep

    def split_device(self, keep: np.ndarray, move: bool, d_keys: Optional[int], d_vals: Optional[int],
                     capacity: int) -> int:
        """gd_dir_split_device; d_keys None = size query.  Returns the entries selected."""
        keep = np.ascontiguousarray(keep, dtype=np.uint8)
        n = C.c_uint64(0)
        self._c(lib.gd_dir_split_device(self.h, _ptr(keep), len(keep), 1 if move else 0,
                                        C.c_void_p(d_keys) if d_keys else None,
                                        C.c_void_p(d_vals) if d_vals else None, capacity, C.byref(n)))
        return n.value

    def rehash(self, capacity: int):
        self._c(lib.gd_dir_rehash(self.h, capacity))

    # -- hot path (host arrays) --------------------------------------------------
    def route(self, keys):
        k = keys_array(keys)
        n = len(k)
        silo = np.zeros(n, dtype=np.uint32)
        act = np.zeros(n, dtype=np.uint32)
        st = np.zeros(n, dtype=np.uint8)
        self._c(lib.gd_route(self.h, _ptr(k), n, _ptr(silo), _ptr(act), _ptr(st)))
        return st, silo, act

    def bucket(self, acts, n_act: int):
        a = np.ascontiguousarray(np.asarray(acts, dtype=np.uint32))
        perm = np.zeros(len(a), dtype=np.uint32)
        off = np.zeros(n_act + 2, dtype=np.uint32)
        self._c(lib.gd_bucket(self.h, _ptr(a), len(a), n_act, _ptr(perm), _ptr(off)))
        return perm, off

    def route_bucket(self, keys, n_act: int):
        k = keys_array(keys)
        n = len(k)
        silo = np.zeros(n, dtype=np.uint32)
        act = np.zeros(n, dtype=np.uint32)
        st = np.zeros(n, dtype=np.uint8)
        perm = np.zeros(n, dtype=np.uint32)
        off = np.zeros(n_act + 2, dtype=np.uint32)
        self._c(lib.gd_route_bucket(self.h, _ptr(k), n, n_act, _ptr(silo), _ptr(act), _ptr(st), _ptr(perm), _ptr(off)))
        return st, silo, act, perm, off

    # -- KeyExt grains (string keys, compound keys, geo clients) ------------------------
    @staticmethod
    def _ext(exts, n: int) -> KeyExtBatch:
        x = exts if isinstance(exts, KeyExtBatch) else KeyExtBatch(list(exts))
        assert len(x.length) == n, "one KeyExt entry per key"
        return x

    def register_ext(self, keys, exts, acts, silos):
        k = keys_array(keys)
        n = len(k)
        x = self._ext(exts, n)
        vals = np.zeros((n, 2), dtype=np.uint32)
        vals[:, 0] = acts
        vals[:, 1] = silos
        out = np.zeros((n, 2), dtype=np.uint32)
        ins = np.zeros(n, dtype=np.uint8)
        self._c(lib.gd_dir_register_ext(self.h, _ptr(k), C.byref(x.struct), _ptr(vals), n, _ptr(out), _ptr(ins)))
        return out[:, 0].copy(), out[:, 1].copy(), ins

    def unregister_ext(self, keys, exts, acts) -> np.ndarray:
        k = keys_array(keys)
        n = len(k)
        x = self._ext(exts, n)
        a = np.ascontiguousarray(acts, dtype=np.uint32)
        out = np.zeros(n, dtype=np.uint8)
        self._c(lib.gd_dir_unregister_ext(self.h, _ptr(k), C.byref(x.struct), _ptr(a), n, _ptr(out)))
        return out

    def lookup_ext(self, keys, exts):
        k = keys_array(keys)
        n = len(k)
        x = self._ext(exts, n)
        vals = np.zeros((n, 2), dtype=np.uint32)
        found = np.zeros(n, dtype=np.uint8)
        self._c(lib.gd_dir_lookup_ext(self.h, _ptr(k), C.byref(x.struct), n, _ptr(vals), _ptr(found)))
        return found, vals[:, 0].copy(), vals[:, 1].copy()

    def uniform_hashes_ext(self, keys, exts) -> np.ndarray:
        k = keys_array(keys)
        n = len(k)
        x = self._ext(exts, n)
        out = np.zeros(n, dtype=np.uint32)
        self._c(lib.gd_uniform_hashes_ext(self.h, _ptr(k), C.byref(x.struct), n, _ptr(out)))
        return out

    def ext_stats(self) -> dict:
        live, cap, heap = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self._c(lib.gd_dir_ext_stats(self.h, C.byref(live), C.byref(cap), C.byref(heap)))
        return {"live": live.value, "capacity": cap.value, "heap_bytes": heap.value}

    def route_ext(self, keys, exts):
        k = keys_array(keys)
        n = len(k)
        x = self._ext(exts, n)
        silo = np.zeros(n, dtype=np.uint32)
        act = np.zeros(n, dtype=np.uint32)
        st = np.zeros(n, dtype=np.uint8)
        self._c(lib.gd_route_ext(self.h, _ptr(k), C.byref(x.struct), n, _ptr(silo), _ptr(act), _ptr(st)))
        return st, silo, act

    def route_bucket_ext(self, keys, exts, n_act: int):
        k = keys_array(keys)
        n = len(k)
        x = self._ext(exts, n)
        silo = np.zeros(n, dtype=np.uint32)
        act = np.zeros(n, dtype=np.uint32)
        st = np.zeros(n, dtype=np.uint8)
        perm = np.zeros(n, dtype=np.uint32)
        off = np.zeros(n_act + 2, dtype=np.uint32)
        self._c(lib.gd_route_bucket_ext(self.h, _ptr(k), C.byref(x.struct), n, n_act, _ptr(silo), _ptr(act), _ptr(st),
                                        _ptr(perm), _ptr(off)))
        return st, silo, act, perm, off

    def route_bucket_ext_device(self, d_keys: int, d_bytes: int, d_offset: int, d_length: int, bytes_len: int, n: int,
                                n_act: int, d_silo: int, d_act: int, d_status: int, d_perm: int, d_offsets: int):
        dx = gd_key_ext(d_bytes, d_offset, d_length, bytes_len)
        self._c(lib.gd_route_bucket_ext_device(self.h, C.c_void_p(d_keys), C.byref(dx), n, n_act, C.c_void_p(d_silo),
                                               C.c_void_p(d_act), C.c_void_p(d_status), C.c_void_p(d_perm),
                                               C.c_void_p(d_offsets)))

    # -- non-owner directory cache -------------------------------------
    @staticmethod
    def _silo_mask(silos, n_silos: int, default: int) -> np.ndarray:
        m = np.full(max(n_silos, 1), default, dtype=np.uint8)
        if silos is not None:
            m[:] = 0
            m[[int(x) for x in silos]] = 1
        return m

    def cache_configure(self, max_size: int, local_silos, n_silos: int, valid_silos=None):
        """LocalLookup mode: grains owned by `local_silos` are probed here, the rest in an
        LRU cache of `max_size` entries (valid_silos None = every silo valid)."""
        loc = self._silo_mask(local_silos, n_silos, 0)
        val = self._silo_mask(valid_silos, n_silos, 1)
        self._c(lib.gd_cache_configure(self.h, max_size, _ptr(loc), _ptr(val), n_silos))

    def cache_set_silos(self, local_silos, n_silos: int, valid_silos=None):
        loc = self._silo_mask(local_silos, n_silos, 0)
        val = self._silo_mask(valid_silos, n_silos, 1)
        self._c(lib.gd_cache_set_silos(self.h, _ptr(loc), _ptr(val), n_silos))

    def cache_add(self, keys, acts, silos, versions, exts=None):
        """AddOrUpdate in order; exts (one per key, see KeyExtBatch) keys KeyExt grains by their string."""
        k = keys_array(keys)
        n = len(k)
        vals = np.zeros((n, 2), dtype=np.uint32)
        vals[:, 0] = acts
        vals[:, 1] = silos
        ver = np.ascontiguousarray(np.asarray(versions, dtype=np.int32))
        if exts is None:
            self._c(lib.gd_cache_add(self.h, _ptr(k), _ptr(vals), _ptr(ver), n))
        else:
            x = self._ext(exts, n)
            self._c(lib.gd_cache_add_ext(self.h, _ptr(k), C.byref(x.struct), _ptr(vals), _ptr(ver), n))

    def cache_remove(self, keys, exts=None) -> np.ndarray:
        k = keys_array(keys)
        out = np.zeros(len(k), dtype=np.uint8)
        if exts is None:
            self._c(lib.gd_cache_remove(self.h, _ptr(k), len(k), _ptr(out)))
        else:
            x = self._ext(exts, len(k))
            self._c(lib.gd_cache_remove_ext(self.h, _ptr(k), C.byref(x.struct), len(k), _ptr(out)))
        return out

    def cache_lookup(self, keys, exts=None):
        """Returns (found u8, act u32, silo u32, version i32)."""
        k = keys_array(keys)
        n = len(k)
        vals = np.zeros((n, 2), dtype=np.uint32)
        ver = np.zeros(n, dtype=np.int32)
        found = np.zeros(n, dtype=np.uint8)
        if exts is None:
            self._c(lib.gd_cache_lookup(self.h, _ptr(k), n, _ptr(vals), _ptr(ver), _ptr(found)))
        else:
            x = self._ext(exts, n)
            self._c(lib.gd_cache_lookup_ext(self.h, _ptr(k), C.byref(x.struct), n, _ptr(vals), _ptr(ver),
                                            _ptr(found)))
        return found, vals[:, 0].copy(), vals[:, 1].copy(), ver

    def cache_clear(self):
        self._c(lib.gd_cache_clear(self.h))

    def cache_stats(self) -> dict:
        s = gd_cache_stats()
        self._c(lib.gd_cache_stats_get(self.h, C.byref(s)))
        return {name: int(getattr(s, name)) for name, _ in gd_cache_stats._fields_}

    def cache_entries(self) -> dict:
        """key tuple -> (act, silo, version, generation)."""
        n = C.c_uint64(0)
        self._c(lib.gd_cache_entries(self.h, None, None, None, None, 0, C.byref(n)))
        m = n.value
        k = np.zeros((max(m, 1), 3), dtype=np.uint64)
        v = np.zeros((max(m, 1), 2), dtype=np.uint32)
        ver = np.zeros(max(m, 1), dtype=np.int32)
        gen = np.zeros(max(m, 1), dtype=np.uint64)
        if m:
            self._c(lib.gd_cache_entries(self.h, _ptr(k), _ptr(v), _ptr(ver), _ptr(gen), m, C.byref(n)))
        return {tuple(int(x) for x in k[i]): (int(v[i, 0]), int(v[i, 1]), int(ver[i]), int(gen[i]))
                for i in range(m)}

    def cache_entries_ext(self) -> dict:
        """(n0, n1, tcd) or (n0, n1, tcd, KeyExt bytes) -> (act, silo, version, generation)."""
        n, nb = C.c_uint64(0), C.c_uint64(0)
        self._c(lib.gd_cache_entries_ext(self.h, None, None, None, None, None, None, None, 0, 0, C.byref(n),
                                         C.byref(nb)))
        m, b = n.value, nb.value
        k = np.zeros((max(m, 1), 3), dtype=np.uint64)
        v = np.zeros((max(m, 1), 2), dtype=np.uint32)
        ver = np.zeros(max(m, 1), dtype=np.int32)
        gen = np.zeros(max(m, 1), dtype=np.uint64)
        xl = np.zeros(max(m, 1), dtype=np.int32)
        xo = np.zeros(max(m, 1), dtype=np.uint64)
        blob = np.zeros(max(b, 1), dtype=np.uint8)
        if m:
            self._c(lib.gd_cache_entries_ext(self.h, _ptr(k), _ptr(v), _ptr(ver), _ptr(gen), _ptr(xl), _ptr(xo),
                                             _ptr(blob), m, b, C.byref(n), C.byref(nb)))
        out = {}
        for i in range(m):
            key = tuple(int(x) for x in k[i])
            if xl[i] >= 0:
                key = key + (bytes(blob[int(xo[i]):int(xo[i]) + int(xl[i])]),)
            out[key] = (int(v[i, 0]), int(v[i, 1]), int(ver[i]), int(gen[i]))
        return out

    # -- follower fan-out ----------------------------------------------
    def fanout_route_bucket(self, row_off, dst, frontier, type_code: int, n_act: Optional[int]):
        """One publish hop (gd_fanout_route_bucket): returns dict of target, sender, status,
        silo, act (+ perm, offsets when n_act is not None)."""
        ro = np.ascontiguousarray(np.asarray(row_off, dtype=np.uint32))
        d = np.ascontiguousarray(np.asarray(dst, dtype=np.uint32))
        if d.size == 0:
            d = np.zeros(1, dtype=np.uint32)
        fr = np.ascontiguousarray(np.asarray(frontier, dtype=np.uint32))
        n_nodes = len(ro) - 1
        n = C.c_uint64(0)
        na = 0 if n_act is None else n_act
        # size query through the fused call with capacity 0 would do the work twice: count on the host
        valid = fr[fr < n_nodes]
        m = int((ro[valid.astype(np.int64) + 1].astype(np.int64) - ro[valid].astype(np.int64)).sum())
        out = {k: np.zeros(m, dtype=np.uint32) for k in ("target", "sender", "silo", "act")}
        out["status"] = np.zeros(m, dtype=np.uint8)
        perm = off = None
        if n_act is not None:
            perm = np.zeros(m, dtype=np.uint32)
            off = np.zeros(na + 2, dtype=np.uint32)
        P = lambda a: None if a is None else _ptr(a)  # noqa: E731
        self._c(lib.gd_fanout_route_bucket(self.h, _ptr(ro), _ptr(d), n_nodes, _ptr(fr) if len(fr) else None, len(fr),
                                           type_code, na, P(out["target"]), P(out["sender"]), P(out["silo"]),
                                           P(out["act"]), P(out["status"]), P(perm), P(off), m, C.byref(n)))
        assert n.value == m
        if n_act is not None:
            out["perm"], out["offsets"] = perm, off
        return out

    def fanout_expand_device(self, d_row_off: int, d_dst: int, n_nodes: int, d_frontier: int, n_frontier: int,
                             d_target: Optional[int], d_sender: Optional[int], capacity: int) -> int:
        n = C.c_uint64(0)
        self._c(lib.gd_fanout_expand_device(self.h, d_row_off, d_dst, n_nodes, d_frontier, n_frontier,
                                            d_target or None, d_sender or None, capacity, C.byref(n)))
        return n.value

    def fanout_route_bucket_device(self, d_row_off: int, d_dst: int, n_nodes: int, d_frontier: int, n_frontier: int,
                                   type_code: int, n_act: int, d_target: Optional[int], d_sender: int, d_silo: int,
                                   d_act: int, d_status: int, d_perm: Optional[int], d_offsets: Optional[int],
                                   capacity: int) -> int:
        n = C.c_uint64(0)
        self._c(lib.gd_fanout_route_bucket_device(self.h, d_row_off, d_dst, n_nodes, d_frontier, n_frontier, type_code,
                                                  n_act, d_target or None, d_sender, d_silo, d_act, d_status,
                                                  d_perm or None, d_offsets or None, capacity, C.byref(n)))
        return n.value

    def route_nodes_device(self, d_nodes: int, n: int, type_code: int, d_silo: int, d_act: int, d_status: int):
        self._c(lib.gd_route_nodes_device(self.h, d_nodes, n, type_code, d_silo, d_act, d_status))

    def pack_nodes_by_shard_device(self, d_nodes: int, d_payload: int, n: int, type_code: int, n_shards: int,
                                   d_send_nodes: int, d_send_payload: int, d_counts: int):
        self._c(lib.gd_pack_nodes_by_shard_device(self.h, d_nodes, d_payload, n, type_code, n_shards, d_send_nodes,
                                                  d_send_payload, d_counts))

    def frontier_next_device(self, d_offsets: int, n_act: int, d_visited: int, d_out: int) -> int:
        n = C.c_uint32(0)
        self._c(lib.gd_frontier_next_device(self.h, d_offsets, n_act, d_visited, d_out, C.byref(n)))
        return n.value

    # -- hot path (device pointers; enqueue only) -----------------------------------
    def route_device(self, d_keys: int, n: int, d_silo: int, d_act: int, d_status: int):
        self._c(lib.gd_route_device(self.h, C.c_void_p(d_keys), n, C.c_void_p(d_silo), C.c_void_p(d_act),
                                    C.c_void_p(d_status)))

    def route_bound_device(self, d_keys: int, n: int, d_silo: int, d_act: int, d_status: int):
        """gd_route_bound_device (diagnostic): the route kernel's memory bound over the 8-B index; the
        outputs are not route results."""
        self._c(lib.gd_route_bound_device(self.h, C.c_void_p(d_keys), n, C.c_void_p(d_silo), C.c_void_p(d_act),
                                          C.c_void_p(d_status)))

    def bucket_device(self, d_acts: int, n: int, n_act: int, d_perm: int, d_offsets: int):
        self._c(lib.gd_bucket_device(self.h, C.c_void_p(d_acts), n, n_act, C.c_void_p(d_perm), C.c_void_p(d_offsets)))

    def route_bucket_device(self, d_keys: int, n: int, n_act: int, d_silo: int, d_act: int, d_status: int,
                            d_perm: int, d_offsets: int):
        self._c(lib.gd_route_bucket_device(self.h, C.c_void_p(d_keys), n, n_act, C.c_void_p(d_silo),
                                           C.c_void_p(d_act), C.c_void_p(d_status), C.c_void_p(d_perm),
                                           C.c_void_p(d_offsets)))

    def ring_owner_device(self, d_keys: int, n: int, d_silo: int):
        self._c(lib.gd_ring_owner_device(self.h, C.c_void_p(d_keys), n, C.c_void_p(d_silo)))

    def pack_by_shard_device(self, d_keys: int, n: int, n_shards: int, d_send_keys: int, d_send_idx: int,
                             d_counts: int):
        self._c(lib.gd_pack_by_shard_device(self.h, C.c_void_p(d_keys), n, n_shards, C.c_void_p(d_send_keys),
                                            C.c_void_p(d_send_idx), C.c_void_p(d_counts)))

    def pack_routes_by_rank_device(self, d_keys: int, d_status: int, d_silo: int, n: int, n_shards: int, my_rank: int,
                                   d_send_keys: int, d_send_pos: int, d_counts: int):
        self._c(lib.gd_pack_routes_by_rank_device(self.h, C.c_void_p(d_keys), C.c_void_p(d_status), C.c_void_p(d_silo),
                                                  n, n_shards, my_rank, C.c_void_p(d_send_keys),
                                                  C.c_void_p(d_send_pos), C.c_void_p(d_counts)))

    # -- in-library exchange over RCCL (SURVEY 8 b gd_route_multi, 8 e) ----------------
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = (C.c_uint8 * GD_COMM_ID_BYTES)()
        _check(None, lib.gd_comm_unique_id(buf))
        return bytes(buf)

    def comm_init(self, unique_id: bytes, n_ranks: int, rank: int):
        assert len(unique_id) == GD_COMM_ID_BYTES
        buf = (C.c_uint8 * GD_COMM_ID_BYTES).from_buffer_copy(unique_id)
        self._c(lib.gd_comm_init(self.h, buf, n_ranks, rank))

    @staticmethod
    def comm_init_local(engines: Sequence["GrainDispatch"]):
        """gd_comm_init_local: the engines become ranks 0..W-1 of an in-process communicator (the
        W > 1 exchange rehearsed on one GPU; drive each engine from its own thread)."""
        arr = (C.c_void_p * len(engines))(*[e.h.value for e in engines])
        _check(None, lib.gd_comm_init_local(arr, len(engines)))

    def comm_destroy(self):
        self._c(lib.gd_comm_destroy(self.h))

    def route_multi_device(self, d_keys: int, n: int, n_act: int, return_routes: bool = False,
                           keys_ready: bool = False, forward: bool = False,
                           no_keys: bool = False) -> gd_multi_result:
        """Returns after the counts round; the rest is enqueued.  The result holds device pointers
        into library-owned buffers, valid through the next call (two batches in flight)."""
        r = gd_multi_result()
        flags = ((GD_MULTI_RETURN_ROUTES if return_routes else 0) | (GD_MULTI_KEYS_READY if keys_ready else 0)
                 | (GD_MULTI_FORWARD if forward else 0) | (GD_MULTI_NO_KEYS if no_keys else 0))
        self._c(lib.gd_route_multi_device(self.h, C.c_void_p(d_keys), n, n_act, flags, C.byref(r)))
        return r

    def route_multi(self, keys, n_act: int, return_routes: bool = False, forward: bool = False,
                    no_keys: bool = False) -> dict:
        """Host batch in, host results out (gd_route_multi + gd_multi_fetch)."""
        k = keys_array(keys)
        n = k.shape[0]
        r = gd_multi_result()
        flags = ((GD_MULTI_RETURN_ROUTES if return_routes else 0) | (GD_MULTI_FORWARD if forward else 0)
                 | (GD_MULTI_NO_KEYS if no_keys else 0))
        self._c(lib.gd_route_multi(self.h, _ptr(k), n, n_act, flags, C.byref(r)))
        return self.multi_fetch(r, n)

    # -- sharded fan-out cascade (gd_fanout_multi*) ------------------------------------
    def fanout_multi_device(self, d_row_off: int, d_dst: int, n_nodes: int, d_seeds: int, n_seeds: int,
                            type_code: int, n_act: int, hops: int):
        """gd_fanout_multi_device (collective over the communicator): a list of gd_fanout_hop with
        device pointers into library-owned buffers, valid until the next call."""
        out = (gd_fanout_hop * hops)()
        self._c(lib.gd_fanout_multi_device(self.h, C.c_void_p(d_row_off), C.c_void_p(d_dst), n_nodes,
                                           C.c_void_p(d_seeds or 0), n_seeds, type_code, n_act, hops, out))
        return list(out)

    def fanout_multi_part_device(self, d_row_off: int, d_dst: int, n_rows: int, d_node_of: int, d_seeds: int,
                                 n_seeds: int, type_code: int, hops: int):
        """gd_fanout_multi_part_device (collective): the cascade over this rank's partition of the
        follower graph (row i = local activation i, node d_node_of[i]); gd_fanout_hop list as
        fanout_multi_device (offsets over the n_rows local activations)."""
        out = (gd_fanout_hop * hops)()
        self._c(lib.gd_fanout_multi_part_device(self.h, C.c_void_p(d_row_off), C.c_void_p(d_dst or 0), n_rows,
                                                C.c_void_p(d_node_of or 0), C.c_void_p(d_seeds or 0), n_seeds,
                                                type_code, hops, out))
        return list(out)

    def fanout_cascade_device(self, d_row_off: int, d_dst: int, n_nodes: int, d_seeds: int, n_seeds: int,
                              type_code: int, n_act: int, hops: int):
        """gd_fanout_cascade_device: the one-GPU cascade inside the library; gd_fanout_hop list (device
        pointers into library buffers, src NULL), hops copied out with fanout_multi_fetch."""
        out = (gd_fanout_hop * hops)()
        self._c(lib.gd_fanout_cascade_device(self.h, C.c_void_p(d_row_off), C.c_void_p(d_dst or 0), n_nodes,
                                             C.c_void_p(d_seeds or 0), n_seeds, type_code, n_act, hops, out))
        return list(out)

    def fanout_multi(self, row_off, dst, seeds, type_code: int, n_act: int, hops: int) -> List[dict]:
        """gd_fanout_multi (host graph and seeds) + gd_fanout_multi_fetch of every hop."""
        ro = np.ascontiguousarray(row_off, dtype=np.uint32)
        d = np.ascontiguousarray(dst, dtype=np.uint32)
        sd = np.ascontiguousarray(seeds, dtype=np.uint32)
        out = (gd_fanout_hop * hops)()
        self._c(lib.gd_fanout_multi(self.h, _ptr(ro), _ptr(d) if d.size else None, len(ro) - 1,
                                    _ptr(sd) if sd.size else None, sd.size, type_code, n_act, hops, out))
        return [self.fanout_multi_fetch(i, out[i], n_act) for i in range(hops)]

    def fanout_multi_fetch(self, hop: int, r: gd_fanout_hop, n_act: int) -> dict:
        m = r.n_recv
        res = {"frontier": np.empty(r.n_frontier, np.uint32), "target": np.empty(m, np.uint32),
               "sender": np.empty(m, np.uint32), "src": np.empty(m, np.uint32), "silo": np.empty(m, np.uint32),
               "act": np.empty(m, np.uint32), "status": np.empty(m, np.uint8), "perm": np.empty(m, np.uint32),
               "offsets": np.empty(n_act + 2, np.uint32)}
        names = ("frontier", "target", "sender", "src", "silo", "act", "status", "perm", "offsets")
        self._c(lib.gd_fanout_multi_fetch(self.h, hop, *[C.c_void_p(_ptr(res[f])) if res[f].size else None
                                                         for f in names]))
        res["n_sent"] = int(r.n_sent)
        return res

    # -- multi-rank directory handoff (gd_dir_handoff_multi) ----------------------------
    def handoff_multi(self, keep_silos, n_silos: int, event: int, act_base: int) -> dict:
        """gd_dir_handoff_multi (collective) + gd_dir_handoff_fetch: the entries this rank received,
        in arrival order, with their activation index here, status and dropped address."""
        keep = self.keep_mask(keep_silos, n_silos)
        r = gd_handoff_result()
        self._c(lib.gd_dir_handoff_multi(self.h, _ptr(keep), len(keep), event, act_base, C.byref(r)))
        m = r.n_recv
        out = {"keys": np.empty((m, 3), np.uint64), "ids": np.empty((m, 3), np.uint64), "act": np.empty(m, np.uint32),
               "silo": np.empty(m, np.uint32), "src": np.empty(m, np.uint32), "status": np.empty(m, np.uint8),
               "dropped": np.empty((m, 2), np.uint32)}
        names = ("keys", "ids", "act", "silo", "src", "status", "dropped")
        self._c(lib.gd_dir_handoff_fetch(self.h, *[C.c_void_p(_ptr(out[f])) if m else None for f in names]))
        out["n_sent"] = int(r.n_sent)
        return out

    def split_ext(self, keep_silos, n_silos: int, move: bool = True):
        """gd_dir_split_ext: (keys (m,3) u64, acts, silos, KeyExt list (bytes / None)) in slot order."""
        keep = self.keep_mask(keep_silos, n_silos)
        n, nb = C.c_uint64(), C.c_uint64()
        self._c(lib.gd_dir_split_ext(self.h, _ptr(keep), len(keep), int(move), None, None, None, None, None, 0, 0,
                                     C.byref(n), C.byref(nb)))
        m = n.value
        keys = np.zeros((m, 3), np.uint64)
        vals = np.zeros((m, 2), np.uint32)
        off = np.zeros(m, np.uint64)
        ln = np.zeros(m, np.int32)
        blob = np.zeros(max(1, nb.value), np.uint8)
        if m:
            self._c(lib.gd_dir_split_ext(self.h, _ptr(keep), len(keep), int(move), _ptr(keys), _ptr(vals), _ptr(off),
                                         _ptr(ln), _ptr(blob), m, nb.value, C.byref(n), C.byref(nb)))
        exts = [None if ln[i] < 0 else bytes(blob[int(off[i]):int(off[i]) + int(ln[i])]) for i in range(m)]
        return keys, vals[:, 0].copy(), vals[:, 1].copy(), exts

    def ring_owner_ext(self, keys, exts) -> np.ndarray:
        k = keys_array(keys)
        n = len(k)
        x = self._ext(exts, n)
        out = np.zeros(n, dtype=np.uint32)
        self._c(lib.gd_ring_owner_ext(self.h, _ptr(k), C.byref(x.struct), n, _ptr(out)))
        return out

    def route_multi_ext(self, keys, exts, n_act: int, return_routes: bool = False, forward: bool = False) -> dict:
        """route_multi with KeyExt grains routed on their owner (strings travel with the batch)."""
        k = keys_array(keys)
        n = k.shape[0]
        x = self._ext(exts, n)
        r = gd_multi_result()
        flags = (GD_MULTI_RETURN_ROUTES if return_routes else 0) | (GD_MULTI_FORWARD if forward else 0)
        self._c(lib.gd_route_multi_ext(self.h, _ptr(k), C.byref(x.struct), n, n_act, flags, C.byref(r)))
        return self.multi_fetch(r, n)

    def multi_fetch(self, r: gd_multi_result, n: int) -> dict:
        """Host copies of the last gd_route_multi* result (n = this rank's batch size)."""
        m = r.n_recv
        out = {"recv_keys": np.empty((m, 3), np.uint64) if r.recv_keys else None, "recv_idx": np.empty(m, np.uint32),
               "recv_src": np.empty(m, np.uint32), "silo": np.empty(m, np.uint32), "act": np.empty(m, np.uint32),
               "status": np.empty(m, np.uint8), "perm": np.empty(m, np.uint32),
               "offsets": np.empty(r.n_act + 2, np.uint32)}
        if r.ret_silo:
            out.update(ret_silo=np.empty(n, np.uint32), ret_act=np.empty(n, np.uint32), ret_status=np.empty(n, np.uint8))
        names = ("recv_keys", "recv_idx", "recv_src", "silo", "act", "status", "perm", "offsets", "ret_silo",
                 "ret_act", "ret_status")
        self._c(lib.gd_multi_fetch(self.h, *[C.c_void_p(_ptr(out[f])) if out.get(f) is not None else None
                                             for f in names]))
        return out

    # -- header decode -------------------------------------------------
    @staticmethod
    def _frame_host(n: int, fields) -> Tuple[dict, gd_frame_fields]:
        want = set(FRAME_FIELDS) if fields is None else {"flags", "target_grain", *fields}
        arrs = {k: np.zeros((n,) + FRAME_FIELDS[k][1], dtype=FRAME_FIELDS[k][0]) for k in want}
        ff = gd_frame_fields(**{k: (_ptr(a) if n else None) for k, a in arrs.items()})
        return arrs, ff

    def decode_frames(self, buf: bytes, offsets, fields: Optional[Iterable[str]] = None) -> dict:
        """Decode the frames starting at `offsets` in `buf` (host bytes).  Returns a dict of
        numpy arrays named like gd_frame_fields (all fields unless `fields` narrows it)."""
        b = np.frombuffer(buf, dtype=np.uint8) if len(buf) else np.zeros(1, dtype=np.uint8)
        off = np.ascontiguousarray(np.asarray(offsets, dtype=np.uint64))
        n = len(off)
        arrs, ff = self._frame_host(n, fields)
        self._c(lib.gd_decode_frames(self.h, _ptr(b), len(buf), _ptr(off), n, C.byref(ff)))
        return arrs

    def route_frames(self, buf: bytes, offsets, n_act: Optional[int] = None, fields: Optional[Iterable[str]] = (),
                     keyext: bool = False):
        """Decode -> route (-> bucket when n_act is given).  Returns (decoded fields, status,
        silo, act[, perm, offsets]).  keyext: gd_route_frames_ext (KeyExt targets routed too)."""
        b = np.frombuffer(buf, dtype=np.uint8) if len(buf) else np.zeros(1, dtype=np.uint8)
        off = np.ascontiguousarray(np.asarray(offsets, dtype=np.uint64))
        n = len(off)
        arrs, ff = self._frame_host(n, fields)
        silo = np.zeros(n, dtype=np.uint32)
        act = np.zeros(n, dtype=np.uint32)
        st = np.zeros(n, dtype=np.uint8)
        perm = np.zeros(n, dtype=np.uint32) if n_act is not None else None
        offs = np.zeros(n_act + 2, dtype=np.uint32) if n_act is not None else None
        fn = lib.gd_route_frames_ext if keyext else lib.gd_route_frames
        self._c(fn(self.h, _ptr(b), len(buf), _ptr(off), n, n_act or 0, C.byref(ff), _ptr(silo),
                   _ptr(act), _ptr(st), None if perm is None else _ptr(perm), None if offs is None else _ptr(offs)))
        return (arrs, st, silo, act) if n_act is None else (arrs, st, silo, act, perm, offs)

    def decode_frames_device(self, d_buf: int, buf_len: int, d_offsets: int, n: int, d_fields: dict):
        ff = gd_frame_fields(**{k: C.c_void_p(v) for k, v in d_fields.items()})
        self._c(lib.gd_decode_frames_device(self.h, C.c_void_p(d_buf), buf_len, C.c_void_p(d_offsets), n,
                                            C.byref(ff)))

    def route_frames_device(self, d_buf: int, buf_len: int, d_offsets: int, n: int, n_act: int, d_fields: dict,
                            d_silo: int, d_act: int, d_status: int, d_perm: Optional[int], d_offs: Optional[int]):
        ff = gd_frame_fields(**{k: C.c_void_p(v) for k, v in d_fields.items()})
        self._c(lib.gd_route_frames_device(self.h, C.c_void_p(d_buf), buf_len, C.c_void_p(d_offsets), n, n_act,
                                           C.byref(ff), C.c_void_p(d_silo), C.c_void_p(d_act), C.c_void_p(d_status),
                                           C.c_void_p(d_perm or 0), C.c_void_p(d_offs or 0)))

    # -- per-kernel timing ----------------------------------------------------------
    def kernel_times(self) -> dict:
        arr = (gd_kernel_time * 64)()
        n = C.c_uint32(0)
        self._c(lib.gd_kernel_times(self.h, arr, 64, C.byref(n)))
        return {arr[i].name.decode(): (int(arr[i].launches), float(arr[i].total_ms)) for i in range(min(n.value, 64))}

    def set_kernel_timing(self, enable):
        """False / True: off / every launch; 2: the stages only ("stage:bucket")."""
        self._c(lib.gd_set_kernel_timing(self.h, 2 if enable == 2 else (1 if enable else 0)))

    def kernel_times_reset(self):
        self._c(lib.gd_kernel_times_reset(self.h))


class MicroBatch:
    """gd_microbatch: pinned host buffers + a hipGraph per batch size.
    `keys`, `silo`, `act`, `status`, `perm`, `run_start`, `run_act` are numpy views of the
    pinned buffers (no copies); `n_runs` reads the run count of the last run()."""

    def __init__(self, dispatch: GrainDispatch, capacity: int, n_act: int):
        self.gd = dispatch
        self.capacity, self.n_act = capacity, n_act
        mb = C.c_void_p()
        _check(dispatch.h, lib.gd_microbatch_create(dispatch.h, capacity, n_act, C.byref(mb)))
        self.mb = mb
        kp = lib.gd_microbatch_keys(mb)
        self.keys = np.ctypeslib.as_array(C.cast(kp, C.POINTER(C.c_uint64)), shape=(capacity, 3))
        ptrs = [C.c_void_p() for _ in range(7)]
        _check(dispatch.h, lib.gd_microbatch_outputs(mb, *[C.byref(x) for x in ptrs]))
        u32 = lambda p, n: np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_uint32)), shape=(n,))
        self.silo = u32(ptrs[0], capacity)
        self.act = u32(ptrs[1], capacity)
        self.status = np.ctypeslib.as_array(C.cast(ptrs[2], C.POINTER(C.c_uint8)), shape=(capacity,))
        self.perm = u32(ptrs[3], capacity)
        self._n_runs = u32(ptrs[4], 1)
        self.run_start = u32(ptrs[5], capacity + 1)
        self.run_act = u32(ptrs[6], capacity)

    @property
    def n_runs(self) -> int:
        return int(self._n_runs[0])

    def offsets(self) -> np.ndarray:
        """The runs expanded to gd_bucket's offsets[n_act + 2] (for comparison with it)."""
        r = self.n_runs
        out = np.empty(self.n_act + 2, dtype=np.uint32)
        # offsets[a] = start of the first run with activation >= a; empty buckets share it
        starts = np.append(self.run_start[:r], self.run_start[r])
        acts = np.append(self.run_act[:r].astype(np.int64), self.n_act + 1)
        idx = np.searchsorted(acts, np.arange(self.n_act + 2), side="left")
        out[:] = starts[idx]
        return out

    def run(self, n: int, use_graph: bool = True):
        _check(self.gd.h, lib.gd_microbatch_run(self.mb, n, 1 if use_graph else 0))

    def close(self):
        if getattr(self, "mb", None):
            lib.gd_microbatch_destroy(self.mb)
            self.mb = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
