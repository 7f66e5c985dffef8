"""The C-ABI library loads and exports every symbol include/gnnd.h declares; host-only
argument validation (no device work).  CPU only."""
import ctypes
import os
import re

import numpy as np
import pytest

from gnndecode import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, 'include', 'gnnd.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(gnnd_[a-z0-9_]+)\s*\(', src)))


def test_library_present_and_loads():
    assert os.path.exists(_lib.LIB_PATH), 'build libgnnd.so first (make -C gnn-decode_amd)'
    lib = _lib.get()
    assert lib.gnnd_version() == 1


def test_release_library_reads_no_tuning_env():
    """the planner's A/B switches (gnnd_tune_env in gnnd_common.h) are
    compiled into tuning builds only, so the release library's kernel choice -- and its output
    bits -- cannot depend on the caller's environment.  Every knob the sources name is absent
    from the built release .so, and no source calls getenv directly."""
    csrc = os.path.join(ROOT, 'gnn-decode_amd', 'csrc')
    knobs = set()
    for f in os.listdir(csrc):
        src = open(os.path.join(csrc, f)).read()
        knobs |= set(re.findall(r'gnnd_tune_env\("(GNND_[A-Z0-9_]+)"\)', src))
        code = re.sub(r'//[^\n]*', '', src)
        calls = re.findall(r'\bgetenv\s*\(', code)
        assert f == 'gnnd_common.h' or not calls, f'{f} calls getenv outside gnnd_tune_env'
    assert len(knobs) >= 15, knobs
    lib = open(os.path.join(ROOT, 'gnn-decode_amd', 'gnndecode', 'libgnnd.so'), 'rb').read()
    found = sorted(k for k in knobs if k.encode() in lib)
    assert not found, f'tuning knobs compiled into the release library: {found}'


def test_every_header_symbol_is_exported_and_bound():
    lib = _lib.get()
    names = header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), f'{n} declared in gnnd.h but not exported'
    assert sorted(_lib.SIGNATURES) == names, 'ctypes signature table out of sync with gnnd.h'


def test_status_strings():
    for s in range(6):
        assert _lib.status_string(s)
    assert 'unknown' in _lib.status_string(99)


def test_weights_count_and_width():
    lib = _lib.get()
    n = ctypes.c_int64()
    expect = {'v24': 1283, 'qgnni': 62, 'qbp': 0, 'cgnni': 62, 'cbp': 0}
    for name, cnt in expect.items():
        assert lib.gnnd_weights_count(_lib.VARIANT[name], ctypes.byref(n)) == _lib.OK
        assert n.value == cnt
    assert lib.gnnd_weights_count(9, ctypes.byref(n)) == _lib.ERR_INVALID_ARG
    for name in ('nbp', 'v10'):   # per-edge tables: gnnd_decode_weights_count (needs a graph)
        assert lib.gnnd_weights_count(_lib.VARIANT[name], ctypes.byref(n)) == _lib.ERR_UNSUPPORTED
        assert lib.gnnd_decode_weights_count(None, _lib.VARIANT[name], 15, ctypes.byref(n)) == _lib.ERR_INVALID_ARG
    w = lib.gnnd_propagate_width
    assert w(_lib.VARIANT['v24'], 0) == 2 and w(_lib.VARIANT['v24'], 1) == 2
    assert w(_lib.VARIANT['qgnni'], 0) == 1 and w(_lib.VARIANT['qgnni'], 1) == 2
    for v in ('qbp', 'cgnni', 'cbp', 'v10'):
        assert w(_lib.VARIANT[v], 0) == 1 and w(_lib.VARIANT[v], 1) == 1
    assert w(_lib.VARIANT['nbp'], 0) == 2 and w(_lib.VARIANT['nbp'], 1) == 1
    assert w(9, 0) == -1 and w(0, 5) == -1


def test_prepared_counts_with_channel_prior_tables():
    """gnnd_prepared_weights_count[_priors] (host-only): decoder_v2_4 = 1 283 weights + check-MLP
    table + prior header = 7 264; fp64 V24 adds 17 456 per channel-prior table (<= 64) and 34 864 for
    the readout MLP; other
    models / fp32 take no tables."""
    lib = _lib.get()
    n = ctypes.c_int64()
    v24, f32, f64 = _lib.VARIANT['v24'], 0, 1
    for dt in (f32, f64):
        assert lib.gnnd_prepared_weights_count(v24, dt, ctypes.byref(n)) == _lib.OK and n.value == 7264
        assert lib.gnnd_prepared_weights_count_priors(v24, dt, 0, ctypes.byref(n)) == _lib.OK and n.value == 7264
    assert lib.gnnd_prepared_weights_count_priors(v24, f64, 10, ctypes.byref(n)) == _lib.OK
    assert n.value == 7264 + 10 * 17456 + 34864       # (+ the readout MLP's table)
    assert lib.gnnd_prepared_weights_count_priors(v24, f64, 65, ctypes.byref(n)) == _lib.ERR_INVALID_ARG
    assert lib.gnnd_prepared_weights_count_priors(v24, f64, -1, ctypes.byref(n)) == _lib.ERR_INVALID_ARG
    assert lib.gnnd_prepared_weights_count_priors(v24, f32, 1, ctypes.byref(n)) == _lib.ERR_UNSUPPORTED
    assert lib.gnnd_prepared_weights_count_priors(_lib.VARIANT['cgnni'], f32, 1, ctypes.byref(n)) == _lib.ERR_UNSUPPORTED
    # argument checks before any device call
    assert lib.gnnd_prepare_weights_priors(v24, f64, None, None, None, 3, None) == _lib.ERR_INVALID_ARG
    assert lib.gnnd_prepare_weights_priors(v24, f64, None, None, None, 65, None) == _lib.ERR_INVALID_ARG
    assert lib.gnnd_v24_var_mlp_table(None, None, None, None, None, 4, None) == _lib.ERR_INVALID_ARG
    assert lib.gnnd_v24_var_mlp_table(ctypes.c_void_p(8), None, None, None, None, 4, None) == _lib.ERR_INVALID_ARG


def _graph_create(v, c, V, C):
    lib = _lib.get()
    v = np.ascontiguousarray(v, np.int64)
    c = np.ascontiguousarray(c, np.int64)
    h = ctypes.c_void_p()
    st = lib.gnnd_graph_create(v.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                               c.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                               v.size, V, C, ctypes.byref(h))
    return st, h


@pytest.mark.parametrize('v,c,V,C,status', [
    ([0, 0, 1], [1, 0, 0], 2, 2, _lib.ERR_GRAPH),     # not sorted by (v, c)
    ([0, 0, 1], [0, 0, 1], 2, 2, _lib.ERR_GRAPH),     # duplicate edge
    ([0, 2], [0, 0], 2, 2, _lib.ERR_GRAPH),           # variable out of range
    ([0, 1], [0, -1], 2, 2, _lib.ERR_GRAPH),          # negative check
    ([], [], 2, 2, _lib.ERR_INVALID_ARG),             # empty
    ([0], [0], 0, 2, _lib.ERR_INVALID_ARG),           # no variables
    ([0], [0], 70000, 2, _lib.ERR_UNSUPPORTED),       # beyond 16-bit packing
])
def test_graph_create_rejects_bad_graphs_before_any_device_call(v, c, V, C, status):
    st, h = _graph_create(v, c, V, C)
    assert st == status
    assert not h.value


def test_null_argument_checks():
    lib = _lib.get()
    assert lib.gnnd_graph_destroy(None) == _lib.ERR_INVALID_ARG
    assert lib.gnnd_graph_dims(None, None) == _lib.ERR_INVALID_ARG
    assert lib.gnnd_decode(None, 0, 0, None, None, None, 1, 1, None) == _lib.ERR_INVALID_ARG
    b0 = ctypes.c_int64()
    assert lib.gnnd_train_tape_bytes(None, 0, 0, 1, 1, ctypes.byref(b0)) == _lib.ERR_INVALID_ARG
    assert lib.gnnd_train_fwd(None, 0, 0, None, None, None, None, 1, 1, None) == _lib.ERR_INVALID_ARG
    assert lib.gnnd_train_bwd(None, 0, 0, None, None, None, None, None, None, None, 0, 1, 1,
                              None) == _lib.ERR_INVALID_ARG
    assert lib.gnnd_propagate_tiled(None, 0, 0, 0, 0, None, None, None, 1, None) == _lib.ERR_INVALID_ARG
    cw, lds = ctypes.c_int32(), ctypes.c_int32()
    assert lib.gnnd_decode_tile(None, 0, 0, ctypes.byref(cw), ctypes.byref(lds)) == _lib.ERR_INVALID_ARG
    b = ctypes.c_int64()
    # generic workspace size is host arithmetic
    assert lib.gnnd_propagate_generic_workspace(0, 1, 0, 0, 100, 40, ctypes.byref(b)) == _lib.OK
    assert b.value == (100 + 40) * 4
    assert lib.gnnd_propagate_generic_workspace(2, 1, 1, 1, 100, 40, ctypes.byref(b)) == _lib.OK
    assert b.value == (100 * 2 + 40 * 3 + 200) * 8      # BP c->v mean: src, src2, agg, agg2, cnt, lm x2
    assert lib.gnnd_propagate_generic_workspace(0, 1, 3, 0, 100, 40, ctypes.byref(b)) == _lib.ERR_INVALID_ARG
    # backward workspace: node accumulator; the BP check steps recompute L, sign, g_Lambda
    assert lib.gnnd_propagate_generic_bwd_workspace(0, 1, 0, 1, 100, 40, ctypes.byref(b)) == _lib.OK
    assert b.value == 40 * 8
    assert lib.gnnd_propagate_generic_bwd_workspace(5, 1, 0, 1, 100, 40, ctypes.byref(b)) == _lib.OK
    assert b.value == (2 * 100 + 3 * 40) * 8
    assert lib.gnnd_propagate_generic_bwd_workspace(5, 0, 0, 0, 100, 40, ctypes.byref(b)) == _lib.OK
    assert b.value == 40 * 4
    assert lib.gnnd_propagate_generic_bwd_workspace(0, 1, 1, 0, 100, 40, ctypes.byref(b)) == _lib.ERR_UNSUPPORTED
