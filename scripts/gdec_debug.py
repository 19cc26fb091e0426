#!/usr/bin/env python3
"""gdec_debug.py -- the GPU stream decoder's coder state after the LL and each
band against the host decoder's (tests/native hc_decode_states), to find the
first band where they part.  Development tool (GPU box)."""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rududu-image-codec_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import torch
    import ric_amd
    import hostcoder as HC
    from oracle import oracle as O
    w, h, q, t = [int(x) for x in sys.argv[1:5]] if len(sys.argv) > 4 else (33, 47, 9, 0)
    port = O.port()
    r = port.encode_ric(ric_amd.synth(w, h, 1, 90), q, t)
    hs = np.zeros(64 * 8, np.uint32)
    L = HC.lib()
    L.hc_decode_states.restype = ctypes.c_long
    L.hc_decode_states.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    rb = np.frombuffer(r, np.uint8).copy()
    nb = L.hc_decode_states(rb.ctypes.data, len(r), w, h, hs.ctypes.data)
    istride = (len(r) + 4095) // 4096 * 4096
    buf = np.zeros(istride, np.uint8)
    buf[:len(r)] = rb
    src = torch.from_numpy(buf).cuda()
    dbg = torch.zeros(1024 + w * h * 2, dtype=torch.int64, device="cuda")
    ric_amd.lib().ric_diag_gdec_dbg.argtypes = [ctypes.c_void_p]
    ric_amd.lib().ric_diag_gdec_dbg(dbg.data_ptr())
    out = torch.zeros((1, h, w), dtype=torch.uint8, device="cuda")
    b = ric_amd.Batch(w, h, 1, slots=1, threads=1)
    try:
        b.decompress_gpu(src, istride, [len(r)], [out])
    except Exception as e:
        print("decode:", e)
    ric_amd.lib().ric_diag_gdec_dbg(None)
    gall = dbg.cpu().numpy().view(np.uint32)
    gs = gall[:64 * 8]
    names = ["range", "low", "code", "nbits", "buffer", "p", "ovf", "tag"]
    print("stream %d bytes, %d bands" % (len(r), nb))
    for k in range(nb):
        hv, gv = hs[8 * k:8 * k + 8], gs[8 * k:8 * k + 8]
        same = np.array_equal(hv[:6], gv[:6])
        print("band %2d %s host %s gpu %s" % (k, "ok " if same else "DIFF", list(hv[:7]), list(gv[:7])))
        if not same:
            break
    # every decoded band against the host decoder's (tests/native hc_decode)
    L.hc_decode.restype = ctypes.c_long
    L.hc_decode.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                            ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    pay = np.zeros(len(r) - 9 + 2, np.uint8)
    pay[2:] = rb[9:]
    hb = np.zeros(w * h * 2, np.int32)
    nval = L.hc_decode(pay.ctypes.data, pay.size, 1, w, h, 5, 1, hb.ctypes.data, None)
    gb = gall[2048:2048 + nval].astype(np.uint32).view(np.int32)
    bad = np.nonzero(hb[:nval] != gb)[0]
    print("bands: %d values, %d differ, first %s" % (nval, bad.size, bad[:8]))
    if bad.size:
        k = bad[0]
        print("  host", hb[max(0, k - 4):k + 4], "gpu", gb[max(0, k - 4):k + 4])
    return
    # the decoded LL against the quantised LL (oracle, after buildTree / TSUQ)
    plane = O.gray_plane(ric_amd.synth(w, h, 1, 90)[0] if ric_amd.synth(w, h, 1, 90).ndim == 3 else ric_amd.synth(w, h, 1, 90), q)
    bands = port.bands(plane, stage=1, quant=O.quants(q + 20) if q else 0, lam=O.quants(q + 13) if q else 0)
    ll = np.asarray(bands[-1]).astype(np.int64).ravel()
    gll = gall[1024:1024 + ll.size].astype(np.int32).astype(np.int64)
    bad = np.nonzero(ll[:1024] != gll[:min(1024, ll.size)])[0]
    print("LL %s: %d values, first mismatch %s" % (np.asarray(bands[-1]).shape, ll.size, bad[:5]))
    if bad.size:
        k = bad[0]
        print("  oracle", ll[max(0, k - 3):k + 4], "gpu", gll[max(0, k - 3):k + 4])


if __name__ == "__main__":
    main()
