#!/usr/bin/env python3
"""host_timing.py [W H] -- CPU timing of the product's host serial coder
(record encoder + band decoder, tests/native harness) on one synthetic frame,
bands from the oracle (no GPU).  Development tool."""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from oracle import oracle as O  # noqa: E402
import hostcoder as HC  # noqa: E402
import ctypes  # noqa: E402

W = int(sys.argv[1]) if len(sys.argv) > 1 else 7680
H = int(sys.argv[2]) if len(sys.argv) > 2 else 4320
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
chk = O.port()
pix = O.synth(W, H, 1, 0)
plane = O.gray_plane(pix[0], 9)
bands = chk.bands(plane, stage=1, quant=O.quants(29), lam=O.quants(22))
b = np.ascontiguousarray(np.concatenate([x.ravel() for x in bands]), np.int32)
cap = W * H * 4 + 4096
out = np.zeros(cap, np.uint8)
best_e = best_d = 1e9
for _ in range(reps):
    s1, s2 = ctypes.c_double(), ctypes.c_double()
    n = HC.lib().hc_encode_rec(b.ctypes.data, b.size, 1, W, H, 5, 1, out.ctypes.data, cap, ctypes.byref(s1), ctypes.byref(s2))
    best_e = min(best_e, s1.value)
    buf = out[:n].tobytes()
    dec = np.zeros(b.size, np.int32)
    s = ctypes.c_double()
    src = np.frombuffer(buf, np.uint8).copy()     # keep the copy alive across the call
    HC.lib().hc_decode(src.ctypes.data, len(buf), 1, W, H, 5, 1, dec.ctypes.data, ctypes.byref(s))
    best_d = min(best_d, s.value)
print("bytes %d  encode %.1f ms  decode %.1f ms" % (n, best_e * 1e3, best_d * 1e3))
