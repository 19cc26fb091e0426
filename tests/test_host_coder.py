"""The product's host serial coder (range coder, raw-bit mux, adaptive models,
zerotree scans; csrc/entropy.cpp, encoder.cpp, decoder.cpp) on the CPU,
against the oracle and the golden streams.  Block records are built on the
CPU with the same __host__ __device__ function (csrc/symbols.h) the GPU runs."""
import json
import os

import numpy as np
import pytest

import hostcoder as HC
from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
G = json.load(open(os.path.join(HERE, "golden", "golden.json")))

CASES = [(64, 48, 9, 0, 5, 1), (33, 47, 9, 0, 5, 1), (17, 16, 0, 1, 5, 1), (129, 77, 1, 1, 5, 1),
         (1001, 603, 0, 1, 5, 1), (1000, 600, 5, 0, 5, 1), (512, 512, 0, 1, 3, -1), (121, 45, 0, 1, 5, 1),
         (37, 37, 0, 1, 5, 1), (101, 57, 0, 1, 5, 1), (256, 200, 31, 0, 5, 1), (300, 300, 20, 1, 4, 2)]


def _plane(w, h, q):
    return O.gray_plane(O.synth(w, h, 1, 0)[0], q)


@pytest.mark.parametrize("w,h,q,t,L,lc", CASES)
@pytest.mark.parametrize("records", [True, False])
def test_encode_matches_oracle(w, h, q, t, L, lc, records):
    P = O.port()
    pl = _plane(w, h, q)
    Q = O.quants(q + 20) if q else 0
    lam = O.quants(q + 13) if q else 0
    flat = np.concatenate([x.ravel() for x in P.bands(pl, L, lc, t, 1, Q, lam)]).astype(np.int32)
    assert HC.encode(flat, w, h, L, lc, records) == P.encode_planes(pl[None], L, lc, t, [Q], [lam])


@pytest.mark.parametrize("w,h,q,t,L,lc", CASES)
@pytest.mark.parametrize("nthreads", [0, 3])
def test_split_encoder_matches_oracle(w, h, q, t, L, lc, nthreads):
    """the band-parallel split (events per band, serial replay) writes the
    reference's bytes: raw fields never move across a bin, and bins replay in
    order (muxcodec.cpp:63-74, 536-570)"""
    P = O.port()
    pl = _plane(w, h, q)
    Q = O.quants(q + 20) if q else 0
    lam = O.quants(q + 13) if q else 0
    flat = np.concatenate([x.ravel() for x in P.bands(pl, L, lc, t, 1, Q, lam)]).astype(np.int32)
    assert HC.encode_split(flat, w, h, L, lc, nthreads) == P.encode_planes(pl[None], L, lc, t, [Q], [lam])


@pytest.mark.parametrize("w,h,q,t,L,lc", CASES)
def test_compact_encoder_matches_oracle(w, h, q, t, L, lc):
    """the host walk over the compacted payload (values in walk order, int
    bands dense) writes the reference's bytes"""
    P = O.port()
    pl = _plane(w, h, q)
    Q = O.quants(q + 20) if q else 0
    lam = O.quants(q + 13) if q else 0
    flat = np.concatenate([x.ravel() for x in P.bands(pl, L, lc, t, 1, Q, lam)]).astype(np.int32)
    assert HC.encode_compact(flat, w, h, L, lc) == P.encode_planes(pl[None], L, lc, t, [Q], [lam])


def test_split_encoder_long_raw_fields():
    """lossless int bands: raw fields past 24 bits and events split at 32 bits"""
    P = O.port()
    w, h = 300, 200
    rng = np.random.default_rng(5)
    pl = rng.integers(-2048, 2048, (h, w)).astype(np.int16)
    flat = np.concatenate([x.ravel() for x in P.bands(pl, 5, 4, 1, 1, 0, 0)]).astype(np.int32)
    exp = P.encode_planes(pl[None], 5, 4, 1, [0], [0])
    assert HC.encode(flat, w, h, 5, 4) == exp
    assert HC.encode_split(flat, w, h, 5, 4, 2) == exp


@pytest.mark.parametrize("w,h,q,t,L,lc", CASES)
def test_decode_matches_oracle(w, h, q, t, L, lc):
    P = O.port()
    pl = _plane(w, h, q)
    Q = O.quants(q + 20) if q else 0
    lam = O.quants(q + 13) if q else 0
    buf = P.encode_planes(pl[None], L, lc, t, [Q], [lam])
    _, exp = P.decode_planes(buf, 1, w, h, L, lc, t, [Q], want_bands=True)
    exp = np.concatenate([x.ravel() for x in exp])
    assert np.array_equal(HC.decode(buf, w, h, L, lc, exp.size), exp)


@pytest.mark.parametrize("w,h,q,t,L,lc", CASES)
def test_compact_decoder_matches_oracle(w, h, q, t, L, lc):
    """the finest level decoded into the compacted layout and scattered back
    equals the dense decode (and the oracle's bands)"""
    P = O.port()
    pl = _plane(w, h, q)
    Q = O.quants(q + 20) if q else 0
    lam = O.quants(q + 13) if q else 0
    buf = P.encode_planes(pl[None], L, lc, t, [Q], [lam])
    _, exp = P.decode_planes(buf, 1, w, h, L, lc, t, [Q], want_bands=True)
    exp = np.concatenate([x.ravel() for x in exp])
    assert np.array_equal(HC.decode_compact(buf, w, h, L, lc, exp.size), exp)


def test_c2_full_size_stream():
    e = [x for x in G["large"] if x["name"] == "C2_4096x4096_q9"][0]
    import hashlib
    P = O.port()
    pl = _plane(4096, 4096, 9)
    flat = np.concatenate([x.ravel() for x in P.bands(pl, 5, 1, 0, 1, O.quants(29), O.quants(22))]).astype(np.int32)
    buf = HC.encode(flat, 4096, 4096, 5, 1)
    ric = b"RUD2" + (4096).to_bytes(2, "little") * 2 + bytes([9]) + buf[2:]
    assert hashlib.sha256(ric).hexdigest() == e["ric_sha256"]
    dec = HC.decode(buf, 4096, 4096, 5, 1, flat.size)
    _, exp = P.decode_planes(buf, 1, 4096, 4096, 5, 1, 0, [O.quants(29)], want_bands=True)
    assert np.array_equal(dec, np.concatenate([x.ravel() for x in exp]))


def test_decoder_sanitized_on_hostile_input():
    """The host decoder (csrc/entropy.cpp, decoder.cpp) built with ASan +
    UBSan (tests/native hc_fuzz) on valid, truncated, bit-flipped and garbage
    .ric payloads: no memory error, no undefined behaviour, no hang."""
    import subprocess
    nat = os.path.join(HERE, "native")
    subprocess.run(["make", "-s", "-C", nat, "fuzz"], check=True, capture_output=True, timeout=300)
    files = [os.path.join(HERE, "golden", f) for f in
             ("g17x16_q0_t1_f2.ric", "g33x47_q9_t0_f1.ric", "rgb48x40_q0_t1_f8.ric", "g37x37_q0_t1_f10.ric")]
    r = subprocess.run([os.path.join(nat, "hc_fuzz")] + files, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "runtime error" not in r.stderr and r.stdout.startswith("ok ")
