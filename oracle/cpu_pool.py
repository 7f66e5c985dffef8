"""ORACLE — test/measurement infrastructure only: the all-cores leg of bench.py's
`cpu_baseline` (the CPU restatement timed on every core this host gives us).

bench.py writes a sample of the benchmark batch to an .npz and runs this script as a CHILD
PROCESS (it never forks the GPU process).  This process has not touched the GPU, so it forks
single-threaded workers, each decoding whole chunks with `gnn_oracle.decode`, and prints one
JSON line: {"codewords", "seconds", "workers", "per_worker_s"}.

usage: python oracle/cpu_pool.py SAMPLE.npz WORKERS
  SAMPLE.npz: model (str), T (int), H (uint8 [V, C]), x (float [n_chunks, chunk*N, 1]),
              w/<name> (weights, state_dict names)
"""
import json
import os
import sys
import time

os.environ.setdefault('OMP_NUM_THREADS', '1')
os.environ.setdefault('OPENBLAS_NUM_THREADS', '1')
os.environ.setdefault('MKL_NUM_THREADS', '1')

import numpy as np  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import gnn_oracle  # noqa: E402

_S = {}


def _chunk(k):
    t0 = time.perf_counter()
    gnn_oracle.decode(_S['model'], _S['H'], _S['x'][k], _S['T'], _S['w'])
    return time.perf_counter() - t0


def main():
    path, workers = sys.argv[1], int(sys.argv[2])
    z = np.load(path)
    _S.update(model=str(z['model']), T=int(z['T']), H=z['H'], x=z['x'],
              w={k[2:]: z[k] for k in z.files if k.startswith('w/')})
    n = _S['x'].shape[0]
    N = _S['H'].shape[0] + _S['H'].shape[1]
    import multiprocessing as mp
    ctx = mp.get_context('fork')           # safe: this process never initialised a GPU
    with ctx.Pool(workers) as pool:
        pool.map(_chunk, range(min(workers, n)), chunksize=1)     # page-in, untimed
        t0 = time.perf_counter()
        per = pool.map(_chunk, range(n), chunksize=1)
        wall = time.perf_counter() - t0
    cws = n * (_S['x'].shape[1] // N)
    print(json.dumps({'codewords': cws, 'seconds': wall, 'workers': workers,
                      'per_worker_s': float(np.sum(per)) / workers}), flush=True)


if __name__ == '__main__':
    main()
