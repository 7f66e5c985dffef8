#!/usr/bin/env python3
"""Convert a reference checkpoint (torch.save'd state_dict, possibly CUDA tensors) to .npz.
Reads with torch.load(weights_only=True) only.
usage: python tools/convert_checkpoint.py IN.pkl OUT.npz"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                'gnn-decode_amd'))
from gnndecode import checkpoint  # noqa: E402

if __name__ == '__main__':
    if len(sys.argv) != 3:
        sys.exit(__doc__)
    sd = checkpoint.load_reference(sys.argv[1])
    checkpoint.save_npz(sd, sys.argv[2])
    print(f'{len(sd)} tensors -> {sys.argv[2]}')
