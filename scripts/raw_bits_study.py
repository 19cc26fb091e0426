#!/usr/bin/env python3
"""raw_bits_study.py -- how much of the serial encode pass is raw-bit work
(the question of a GPU pre-pack of the raw bits).

C3 (8K gray q9) stage-1 bands from the oracle, encoded by the product's
record encoder (csrc/encoder.cpp via tests/native): (1) the event counts by
kind (RIC_ENC_STATS build); (2) the pass's time with and without its raw-bit
writes (RIC_ENC_NO_RAW build: wrong output, timing only), median of N runs
on one core."""
import ctypes
import json
import os
import statistics
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import oracle as O  # noqa: E402

NAT = os.path.join(REPO, "tests", "native")


def load(name):
    L = ctypes.CDLL(os.path.join(NAT, name))
    L.hc_encode_rec.restype = ctypes.c_long
    L.hc_encode_rec.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p,
                                ctypes.c_void_p]
    return L


def main():
    subprocess.run(["make", "-s", "-C", NAT, "all", "stats"], check=True)
    W, H, q, reps = 7680, 4320, 9, int(sys.argv[1]) if len(sys.argv) > 1 else 5
    pl = O.gray_plane(O.synth(W, H, 1, 0)[0], q)
    flat = np.concatenate([x.ravel() for x in O.port().bands(pl, 5, 1, 0, 1, O.quants(q + 20), O.quants(q + 13))])
    flat = np.ascontiguousarray(flat, np.int32)
    cap = W * H * 4
    out = np.zeros(cap, np.uint8)
    res = {}
    for name in ("libhostcoder.so", "libhostcoder_stats.so", "libhostcoder_noraw.so"):
        L = load(name)
        ts = []
        for _ in range(reps):
            s1, s2 = ctypes.c_double(), ctypes.c_double()
            n = L.hc_encode_rec(flat.ctypes.data, flat.size, 1, W, H, 5, 1, out.ctypes.data, cap,
                                ctypes.byref(s1), ctypes.byref(s2))
            ts.append(s1.value * 1e3)
        res[name] = {"encode_ms_median": round(statistics.median(ts), 2), "bytes": int(n)}
        if name == "libhostcoder_stats.so":
            st = (ctypes.c_uint64 * 8).in_dll(L, "_ZN3ric11g_enc_statsE")
            k = ["bins", "sign_bits", "remainder_bits", "huffman_bits", "enum_edge_raw_bits", "raw_calls"]
            res["counts_per_frame"] = {k[i]: int(st[i]) // reps for i in range(6)}
    c = res["counts_per_frame"]
    raw = c["sign_bits"] + c["remainder_bits"] + c["huffman_bits"] + c["enum_edge_raw_bits"]
    res["raw_bits_total"] = raw
    res["position_independent_bits"] = c["sign_bits"] + c["enum_edge_raw_bits"]
    res["position_independent_frac"] = round(res["position_independent_bits"] / raw, 4)
    t0 = res["libhostcoder.so"]["encode_ms_median"]
    t1 = res["libhostcoder_noraw.so"]["encode_ms_median"]
    res["raw_bit_share_of_pass"] = round((t0 - t1) / t0, 4)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
