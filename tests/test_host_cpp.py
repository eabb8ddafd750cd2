"""The C++ host layer (orleans_amd/host/orleans_dispatch.hpp) and its tests written
like the reference's (tests/cpp/test_host.cpp): identity tests on CPU; ring,
directory, Dispatcher and IncomingMessageAgent tests on the GPU, plus a routing
dump compared with the oracle."""
import os
import subprocess

import numpy as np
import pytest

import oracle as o

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "build", "test_host")


def _build():
    subprocess.run(["make", "-C", os.path.join(ROOT, "tests", "cpp")], check=True, capture_output=True)
    assert os.path.exists(BIN)


def test_host_cpp_identity_cpu():
    _build()
    p = subprocess.run([BIN, "cpu"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "OK (0 failures)" in p.stdout


@pytest.mark.gpu
def test_host_cpp_gpu(tmp_path):
    _build()
    dump = tmp_path / "route_dump.txt"
    p = subprocess.run([BIN, "all", str(dump)], capture_output=True, text=True, timeout=150)
    assert p.returncode == 0, p.stdout + p.stderr
    for name in ("RingStandalone_Basic", "RingStandalone_Failures", "RingStandalone_Joins", "RingStandalone_Mixed",
                 "VirtualBucketsRanges", "DirectorySemantics", "DispatcherAndAgent", "StringKeyGrains", "MultiActivationGrains", "LruCountTest",
                 "LruMaximumSizeTest", "LruUsageTest", "PerSiloLocalLookup", "PerSiloLocalLookupStringKeys", "WholeNodeExchange", "SiloRemovalAdjustsDirectory",
                 "MergeKeepsLowestActivationId", "MergeStringKeyGrains", "RemoveLastInstanceCountsOnce",
                 "ActivationDirectoryReceive", "RoutingDump"):
        assert f"PASS {name}" in p.stdout, p.stdout + p.stderr
    rows = np.loadtxt(dump, dtype=np.int64)
    tc = o.grain_type_code(o.PING_GRAIN_CLASS)
    keys = o.grain_keys(tc, rows[:, 0])
    spec = o.ring_spec(o.bench_silos(8), "D")
    owner = o.ring_owner_np(spec, o.jenkins_u64x3_np(keys[:, 2], keys[:, 0], keys[:, 1]))
    np.testing.assert_array_equal(rows[:, 1], owner + 1)       # silo 10.0.0.(i+1)
