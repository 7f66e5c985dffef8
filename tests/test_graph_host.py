"""Host-side graph tables (no GPU): every table gnnd_graph_create uploads is rebuilt by
gnnd_graph_validate_host and checked for the invariants the kernels rely on unchecked (slot
plans, padded and x-augmented message layouts), for the framework's codes and random
graphs; the same builder under AddressSanitizer + UBSan (tools/host_sanitize.sh, host code
only) runs clean."""
import ctypes
import os
import shutil
import subprocess

import numpy as np
import pytest

from gnndecode import _lib, codes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _validate(H):
    v, c = (np.ascontiguousarray(a, np.int64) for a in np.nonzero(np.asarray(H)))
    rep = (ctypes.c_int32 * 4)()
    P = ctypes.POINTER(ctypes.c_int64)
    rc = _lib.get().gnnd_graph_validate_host(v.ctypes.data_as(P), c.ctypes.data_as(P), v.size,
                                             H.shape[0], H.shape[1], rep)
    return rc, list(rep)


@pytest.mark.parametrize('code', ['bch_63_45', 'ldpc_648_324', 'toric_4', 'toric_5', 'toric_7'])
def test_code_tables_consistent(code):
    rc, rep = _validate(codes.get_code(code))
    assert rc == _lib.OK and rep[3] == 0 and rep[1] >= 7, rep


def test_random_graph_tables_consistent():
    rng = np.random.default_rng(0)
    for t in range(40):
        V, C = int(rng.integers(1, 300)), int(rng.integers(1, 150))
        H = (rng.random((V, C)) < rng.uniform(0.01, 0.3)).astype(np.uint8)
        H[0, 0] = 1
        rc, rep = _validate(H)
        assert (rc == _lib.OK and rep[3] == 0) or rc == _lib.ERR_UNSUPPORTED, (t, rc, rep)


def test_malformed_edges_rejected():
    P = ctypes.POINTER(ctypes.c_int64)
    v = np.array([1, 0], np.int64)
    c = np.array([0, 0], np.int64)
    assert _lib.get().gnnd_graph_validate_host(v.ctypes.data_as(P), c.ctypes.data_as(P), 2, 2, 1,
                                               None) == _lib.ERR_GRAPH


@pytest.mark.skipif(shutil.which('/opt/rocm/bin/hipcc') is None, reason='hipcc not available')
def test_host_builder_under_asan_ubsan(tmp_path):
    r = subprocess.run(['bash', os.path.join(ROOT, 'tools', 'host_sanitize.sh'), str(tmp_path), '120'],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert 'ERROR: AddressSanitizer' not in r.stderr and 'runtime error' not in r.stderr
    assert '0 bad' in r.stdout
