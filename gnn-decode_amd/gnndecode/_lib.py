"""ctypes binding of libgnnd.so (C ABI declared in include/gnnd.h).

The shared library is built in-tree (`make -C gnn-decode_amd`, or `__graft_entry__.build()`).
There is deliberately no CPU or pure-PyTorch fallback: if the library is missing every
decoder entry point raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('GNND_LIB') or os.path.join(_HERE, 'libgnnd.so')   # GNND_LIB: tuning builds

# enums (include/gnnd.h)
OK, ERR_INVALID_ARG, ERR_HIP, ERR_UNSUPPORTED, ERR_GRAPH, ERR_ALLOC = range(6)
F32, F64, BF16 = 0, 1, 2
SOURCE_TO_TARGET, TARGET_TO_SOURCE = 0, 1
AGGR = {'add': 0, 'mean': 1, 'max': 2}
FLOW = {'source_to_target': SOURCE_TO_TARGET, 'target_to_source': TARGET_TO_SOURCE}
VARIANT = {'v24': 0, 'qgnni': 1, 'qbp': 2, 'cgnni': 3, 'cbp': 4, 'nbp': 5, 'v10': 6, 'v30': 7, 'v22': 8}

_c_i64p = ctypes.POINTER(ctypes.c_int64)
_c_i32p = ctypes.POINTER(ctypes.c_int32)
_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_int = ctypes.c_int

# name -> (restype, argtypes)
SIGNATURES = {
    'gnnd_graph_create': (_int, [_c_i64p, _c_i64p, _i64, _i32, _i32, ctypes.POINTER(_vp)]),
    'gnnd_graph_destroy': (_int, [_vp]),
    'gnnd_graph_validate_host': (_int, [_c_i64p, _c_i64p, _i64, _i32, _i32, _c_i32p]),
    'gnnd_graph_dims': (_int, [_vp, _c_i32p]),
    'gnnd_graph_components': (_int, [_vp, _c_i32p]),
    'gnnd_graph_set_split': (_int, [_vp, _i32]),
    'gnnd_check_tiled': (_int, [_vp, _vp, _i64, _i64, _i64, _i64, _vp, _vp]),
    'gnnd_propagate_width': (_int, [_int, _int]),
    'gnnd_propagate_tiled': (_int, [_vp, _int, _int, _int, _int, _vp, _vp, _vp, _i64, _vp]),
    'gnnd_propagate_generic_workspace': (_int, [_int, _int, _int, _int, _i64, _i64, _c_i64p]),
    'gnnd_propagate_generic': (_int, [_int, _int, _int, _int, _vp, _i64, _i64, _vp, _vp, _i64,
                                      _vp, _vp, _i64, _vp]),
    'gnnd_propagate_tiled_bwd': (_int, [_vp, _int, _int, _int, _int, _vp, _vp, _vp, _vp, _i64,
                                        _vp]),
    'gnnd_propagate_generic_bwd_workspace': (_int, [_int, _int, _int, _int, _i64, _i64, _c_i64p]),
    'gnnd_propagate_generic_bwd': (_int, [_int, _int, _int, _int, _vp, _i64, _i64, _vp, _vp, _vp,
                                          _i64, _vp, _vp, _i64, _vp]),
    'gnnd_weights_count': (_int, [_int, _c_i64p]),
    'gnnd_decode_weights_count': (_int, [_vp, _int, _i32, _c_i64p]),
    'gnnd_prepare_weights': (_int, [_int, _int, _vp, _vp, _vp]),
    'gnnd_prepared_weights_count': (_int, [_int, _int, _c_i64p]),
    'gnnd_prepared_weights_count_priors': (_int, [_int, _int, _i32, _c_i64p]),
    'gnnd_prepare_weights_priors': (_int, [_int, _int, _vp, _vp, ctypes.POINTER(ctypes.c_double), _i32,
                                           _vp]),
    'gnnd_v24_var_mlp_table': (_int, [_vp, _vp, _vp, _vp, _vp, _i64, _vp]),
    'gnnd_decode': (_int, [_vp, _int, _int, _vp, _vp, _vp, _i64, _i32, _vp]),
    'gnnd_decode_tile': (_int, [_vp, _int, _int, _c_i32p, _c_i32p]),
    'gnnd_decode_plan': (_int, [_vp, _int, _int, _c_i32p]),
    'gnnd_train_tape_bytes': (_int, [_vp, _int, _int, _i64, _i32, _c_i64p]),
    'gnnd_train_fwd': (_int, [_vp, _int, _int, _vp, _vp, _vp, _vp, _i64, _i32, _vp]),
    'gnnd_train_bwd_workspace': (_int, [_vp, _int, _int, _i64, _c_i64p]),
    'gnnd_train_workspace_bytes': (_int, [_vp, _int, _int, _i64, _i32, _c_i64p]),
    'gnnd_train_bwd': (_int, [_vp, _int, _int, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64, _i32,
                              _vp]),
    'gnnd_train_bwd_rows': (_int, [_vp, _int, _int, _i64, _c_i64p]),
    'gnnd_train_bwd_partial': (_int, [_vp, _int, _int, _vp, _vp, _vp, _vp, _vp, _vp, _i64, _i64,
                                      _i32, _vp]),
    'gnnd_train_loss_count': (_int, [_vp, _i64, _c_i64p]),
    'gnnd_train_bwd_loss_partial': (_int, [_vp, _int, _int, _vp, _vp, _vp, _vp, _vp, _i32, _i32,
                                           _vp, _vp, _vp, _i64, _i64, _i32, _vp]),
    'gnnd_train_fwd_loss': (_int, [_vp, _int, _int, _vp, _vp, _vp, _vp, _vp, _vp, _i32, _i32,
                                   _vp, _vp, _i64, _i32, _vp]),
    'gnnd_train_update': (_int, [_int, _int, _vp, _i64, _vp, _vp, _i64, _vp, _vp, _vp, _vp, _vp,
                                 _vp, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                 ctypes.c_double, ctypes.c_double, _vp, _vp]),
    'gnnd_syndrome_loss': (_int, [_vp, _vp, _i32, _i32, _int, _vp, _vp, _vp, _vp, _i64, _vp]),
    'gnnd_decision_errors': (_int, [_vp, _vp, _i32, _int, _vp, _vp, _vp, _i64, _vp]),
    'gnnd_v24_check_mlp_table': (_int, [_vp, _vp, _vp, _vp, _i64, _vp, _vp]),
    'gnnd_adam_step': (_int, [_int, _vp, _vp, _vp, _vp, _vp, _i64, ctypes.c_double, ctypes.c_double,
                              ctypes.c_double, ctypes.c_double, ctypes.c_double, _vp]),
    'gnnd_sample_toric': (_int, [_vp, _int, ctypes.POINTER(ctypes.c_double), _i32, ctypes.c_uint64,
                                 _i64, _vp, _vp, _i64, _vp]),
    'gnnd_sample_awgn': (_int, [_vp, _int, ctypes.POINTER(ctypes.c_double), _i32, _vp, _i32, _i32,
                                ctypes.c_uint64, _i64, _vp, _vp, _i64, _vp]),
    'gnnd_philox4x32_10': (None, [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                  ctypes.POINTER(ctypes.c_uint32)]),
    'gnnd_debug_enabled': (_int, []),
    'gnnd_debug_flags': (_int, [ctypes.POINTER(ctypes.c_uint32)]),
    'gnnd_status_string': (ctypes.c_char_p, [_int]),
    'gnnd_last_hip_error': (_int, []),
    'gnnd_version': (_int, []),
}

_lib = None


class GnndError(RuntimeError):
    def __init__(self, fn, status):
        msg = f'{fn} failed: {status_string(status)} (status {status})'
        if status == ERR_HIP:
            msg += f', hipError {get().gnnd_last_hip_error()}'
        super().__init__(msg)
        self.status = status


def get():
    """Load libgnnd.so once; raise ImportError (never fall back) if it is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f'libgnnd.so not found at {LIB_PATH}: build the HIP extension with '
                f'`make -C gnn-decode_amd` (gfx950).  gnndecode has no CPU fallback.')
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def status_string(status):
    return get().gnnd_status_string(status).decode()


def check(fn_name, status):
    if status != OK:
        raise GnndError(fn_name, status)


def call(fn_name, *args):
    check(fn_name, getattr(get(), fn_name)(*args))


def call_or_unsupported(fn_name, *args):
    """call(), except that GNND_ERR_UNSUPPORTED (nothing launched) returns False."""
    status = getattr(get(), fn_name)(*args)
    if status == ERR_UNSUPPORTED:
        return False
    check(fn_name, status)
    return True


def exported_symbols():
    return sorted(SIGNATURES)
