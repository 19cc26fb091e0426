#!/usr/bin/env python3
"""dump_c3.py OUT -- stage-1 (after buildTree) band dump of the C3 frame from
the oracle, int32 canonical order (development tool for hc_main)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from oracle import oracle as O  # noqa: E402

chk = O.port()
pl = O.gray_plane(O.synth(7680, 4320, 1, 0)[0], 9)
b = np.concatenate([x.ravel() for x in chk.bands(pl, stage=1, quant=O.quants(29), lam=O.quants(22))]).astype(np.int32)
b.tofile(sys.argv[1])
