"""band_sums_check.py -- ric_band_sums right after a deferred Transform vs
numpy over the bands read back (debugging the shim's Stats)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "rududu-image-codec_amd")]
import ric_amd
from oracle import oracle as O

w, h = 200, 150
pl = O.gray_plane(ric_amd.synth(w, h, 1, 3)[0], 9)
for order in ("sums_first", "read_first"):
    W = ric_amd.Wavelet2D(w, h, 5, 1)
    W.SetWeight(0)
    W.Transform(pl, w, 0)
    if order == "read_first":
        bands = W.bands()
    got = [W.band_sums(i) for i in range(W.band_count())]
    if order == "sums_first":
        bands = W.bands()
    for i, b in enumerate(bands):
        v = b.astype(np.int64)
        s = int(v.sum())
        ss = int(((v * v) & 0xFFFFFFFF).astype(np.uint32).view(np.int32).astype(np.int64).sum())
        print(order, i, b.shape, "got", got[i], "want", (s, ss), "OK" if got[i] == (s, ss) else "MISMATCH")
