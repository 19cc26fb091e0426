import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "rududu-image-codec_amd"))
import numpy as np
import ric_amd as ric
from oracle import oracle as O
P = O.port()
for (w, h, c, q, t) in [(2048, 24, 1, 17, 0), (96, 80, 3, 5, 0), (96, 80, 1, 5, 0), (256, 256, 1, 17, 0)]:
    pix = ric.synth(w, h, c, w + h)
    r = P.encode_ric(pix, q, t)
    codec = ric.Codec(w, h, c)
    d1, pl1 = codec.decompress(r)
    d0, pl0 = P.decode_ric(r)
    bad = [(p, int((pl1[p] != pl0[p]).sum())) for p in range(c)]
    rows = [np.nonzero((pl1[p] != pl0[p]).any(axis=1))[0][:8].tolist() for p in range(c)]
    print(w, h, c, q, t, "planes mismatch", bad, rows, flush=True)
