"""Single-codeword Tanner graph handle (device-resident CSR/CSC owned by libgnnd).

The reference builds `edge_index = H.to_sparse()._indices()` per codeword and lets PyG
collation tile it with node offsets (quantum/decoder_v2_4.py:161-183; GNNI.forward then
shifts check ids by `rows`, :277).  Every codeword shares H, so `TannerGraph` uploads one
small CSR/CSC once (gnnd_graph_create) and the kernels derive batched ids in closed form.
"""
import ctypes

import numpy as np
import torch

from . import _lib


def edge_list(H):
    """(var, chk) int64 edge list of H[V, C] in `H.to_sparse()._indices()` order."""
    if isinstance(H, torch.Tensor):
        H = H.detach().cpu().numpy()
    H = np.asarray(H)
    v, c = np.nonzero(H)
    return v.astype(np.int64), c.astype(np.int64)


class TannerGraph:
    """Device Tanner graph of one codeword.  `H` is [V, C] (variables x checks)."""

    def __init__(self, H, device=None):
        H = H.detach().cpu().numpy() if isinstance(H, torch.Tensor) else np.asarray(H)
        if H.ndim != 2:
            raise ValueError('H must be a 2-D [V, C] matrix')
        self.V, self.C = int(H.shape[0]), int(H.shape[1])
        self.N = self.V + self.C
        self.H = (H != 0).astype(np.uint8)
        self.var, self.chk = edge_list(self.H)
        self.E = int(self.var.size)
        self.device = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
        lib = _lib.get()
        handle = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            st = lib.gnnd_graph_create(
                self.var.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                self.chk.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                self.E, self.V, self.C, ctypes.byref(handle))
        _lib.check('gnnd_graph_create', st)
        self._handle = handle
        dims = (ctypes.c_int32 * 6)()
        _lib.call('gnnd_graph_dims', handle, dims)
        self.max_var_degree, self.max_chk_degree = int(dims[4]), int(dims[5])
        self._tiled_cache = {}
        from .library import register_graph
        self.gid = register_graph(self)      # id the gnnd:: torch ops take

    @property
    def handle(self):
        return self._handle

    @property
    def components(self):
        """Disconnected components libgnnd split the graph into (1 = not split): decoder_v2_4
        decodes and trains each component of a codeword in its own workgroup."""
        n = ctypes.c_int32()
        _lib.call('gnnd_graph_components', self._handle, ctypes.byref(n))
        return int(n.value)

    def set_split(self, enable):
        """Use (default) or bypass the component split for this graph (A/B and tests)."""
        _lib.call('gnnd_graph_set_split', self._handle, int(bool(enable)))

    def __del__(self):
        h = getattr(self, '_handle', None)
        if h is not None and h.value:
            try:
                _lib.get().gnnd_graph_destroy(h)
            except Exception:
                pass
            self._handle = None

    def __repr__(self):
        return f'TannerGraph(V={self.V}, C={self.C}, E={self.E})'

    # -----------------------------------------------------------------------------------
    def single_edge_index(self, chk_shift=0):
        return torch.from_numpy(np.stack([self.var, self.chk + chk_shift]))

    def batched_edge_index(self, batch, chk_shift=0, device=None):
        """The PyG-collated batch edge_index (node offset b*N), optionally with the
        GNNI.forward check shift (chk_shift = V)."""
        ei = self.single_edge_index(chk_shift).to(device or self.device)
        off = (torch.arange(batch, device=ei.device) * self.N).repeat_interleave(self.E)
        return ei.repeat(1, batch) + off.unsqueeze(0)

    def is_tiled(self, edge_index, chk_shift):
        """True iff `edge_index` is this graph tiled over codewords (checked once per
        tensor/version on the device, cached)."""
        if edge_index.dim() != 2 or edge_index.size(0) != 2 or edge_index.dtype != torch.int64:
            return False
        nE = edge_index.size(1)
        if nE == 0 or nE % self.E:
            return False
        if edge_index.stride(1) != 1:
            return False
        key = (id(edge_index), chk_shift)
        hit = self._tiled_cache.get(key)
        if hit is not None and hit[0]() is edge_index and hit[1] == edge_index._version:
            return hit[2]
        import weakref
        flag = torch.empty(1, dtype=torch.int32, device=edge_index.device)
        _lib.call('gnnd_check_tiled', self._handle, ctypes.c_void_p(edge_index.data_ptr()),
                  edge_index.stride(0), nE, nE // self.E, chk_shift,
                  ctypes.c_void_p(flag.data_ptr()), current_stream(edge_index.device))
        res = bool(flag.item())
        if len(self._tiled_cache) > 64:
            self._tiled_cache.clear()
        self._tiled_cache[key] = (weakref.ref(edge_index), edge_index._version, res)
        return res


def current_stream(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def dtype_code(dtype):
    if dtype == torch.float32:
        return _lib.F32
    if dtype == torch.float64:
        return _lib.F64
    if dtype == torch.bfloat16:
        return _lib.BF16         # storage only (gnnd_decode of the classical models)
    raise TypeError(f'gnndecode kernels support float32/float64 (bf16 storage), got {dtype}')
