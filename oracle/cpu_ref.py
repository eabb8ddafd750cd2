"""ctypes wrapper of oracle/build/libcpuref.so (cpu_ref.c) -- TEST INFRASTRUCTURE ONLY.

The C restatement of the dispatch path, used as bench.py's cpu_baseline
("port") and as an independent cross-check of oracle.py.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "libcpuref.so")


def _load():
    if not os.path.exists(LIB):
        import subprocess
        subprocess.run(["make", "-C", _HERE], check=True, capture_output=True)
    lib = C.CDLL(LIB)
    P, U32, U64 = C.c_void_p, C.c_uint32, C.c_uint64
    lib.cpu_dir_new.restype = P
    lib.cpu_dir_new.argtypes = [C.c_int, U64]
    lib.cpu_dir_free.argtypes = [P]
    lib.cpu_dir_register.argtypes = [P, P, P, P, U64, P, P, P]
    lib.cpu_route.argtypes = [P, C.c_int, C.c_int, P, P, U32, P, U64, U32, U32, P, P, P, C.c_int]
    lib.cpu_bucket.argtypes = [C.c_int, P, U64, U32, P, P, C.c_int]
    lib.cpu_bucket_runs.argtypes = [P, U64, U32, P, P, P, P, P]
    lib.cpu_jenkins_u64x3.restype = U32
    lib.cpu_jenkins_u64x3.argtypes = [U64, U64, U64]
    return lib


lib = _load()
MODES = {"D": 0, "R": 1, "V": 2}


def _p(a):
    return a.ctypes.data


class CpuDirectory:
    def __init__(self, faithful: bool, capacity_hint: int):
        self.faithful = faithful
        self.d = lib.cpu_dir_new(1 if faithful else 0, capacity_hint)

    def __del__(self):
        if getattr(self, "d", None) and lib is not None:
            lib.cpu_dir_free(self.d)
            self.d = None

    def register(self, keys, acts, silos):
        k = np.ascontiguousarray(np.asarray(keys, dtype=np.uint64).reshape(-1, 3))
        a = np.ascontiguousarray(np.asarray(acts, dtype=np.uint32))
        s = np.ascontiguousarray(np.asarray(silos, dtype=np.uint32))
        n = len(k)
        oa = np.zeros(n, np.uint32); os_ = np.zeros(n, np.uint32); oi = np.zeros(n, np.uint8)
        lib.cpu_dir_register(self.d, _p(k), _p(a), _p(s), n, _p(oa), _p(os_), _p(oi))
        return oa, os_, oi

    def route(self, mode, points, owners, keys, my_silo=0, seed_silo=0xFFFFFFFF, nthreads=1):
        pts = np.ascontiguousarray(np.asarray(points, dtype=np.int64).astype(np.uint32))
        own = np.ascontiguousarray(np.asarray(owners, dtype=np.uint32))
        k = np.ascontiguousarray(np.asarray(keys, dtype=np.uint64).reshape(-1, 3))
        n = len(k)
        st = np.zeros(n, np.uint8); silo = np.zeros(n, np.uint32); act = np.zeros(n, np.uint32)
        lib.cpu_route(self.d, 1 if self.faithful else 0, MODES[mode], _p(pts), _p(own), len(pts), _p(k), n,
                      my_silo, seed_silo, _p(st), _p(silo), _p(act), nthreads)
        return st, silo, act


def bucket(acts, n_act, faithful=True, nthreads=1):
    a = np.ascontiguousarray(np.asarray(acts, dtype=np.uint32))
    perm = np.zeros(len(a), np.uint32)
    off = np.zeros(n_act + 2, np.uint32)
    lib.cpu_bucket(1 if faithful else 0, _p(a), len(a), n_act, _p(perm), _p(off), nthreads)
    return perm, off


class BucketRuns:
    """cpu_bucket_runs with its per-activation scratch kept across batches (the micro-batch form:
    the activations present, ascending, each run in arrival order)."""

    def __init__(self, n_act: int, capacity: int):
        self.n_act = n_act
        self.counts = np.zeros(n_act + 1, np.uint32)
        self.perm = np.zeros(capacity, np.uint32)
        self.run_act = np.zeros(capacity, np.uint32)
        self.run_start = np.zeros(capacity + 1, np.uint32)
        self.n_runs = np.zeros(1, np.uint32)

    def __call__(self, acts):
        a = np.ascontiguousarray(np.asarray(acts, dtype=np.uint32))
        lib.cpu_bucket_runs(_p(a), len(a), self.n_act, _p(self.counts), _p(self.perm), _p(self.run_act),
                            _p(self.run_start), _p(self.n_runs))
        r = int(self.n_runs[0])
        return self.perm[:len(a)], self.run_act[:r], self.run_start[:r + 1]
