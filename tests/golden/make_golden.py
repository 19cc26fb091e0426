"""Generate the golden vectors in tests/golden/ from the reference library.

Run in the build container (where /root/reference exists and oracle/Makefile
built oracle/_ref/libricref.so, the unmodified reference sources compiled in
place):   python tests/golden/make_golden.py

Outputs (data only -- inputs and expected outputs):
  *.ric            small .ric files encoded by the reference (CompressImage
                   restated without CImg, oracle/ref_driver.cpp)
  bands_*.npy      canonical band dumps (after Transform / after buildTree)
  golden.json      sha256 of every small .ric and of its decode, plus sha256
                   values of the full-size configs (SURVEY.md §8(c) and
                   BASELINE.json configs) computed by the reference here.
Inputs are the SURVEY.md §8(d) synthetic generator (integer, reproducible).
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from oracle import oracle as O  # noqa: E402

SMALL = [  # (w, h, channels, q, trans, frame)
    (64, 48, 1, 9, 0, 0),
    (33, 47, 1, 9, 0, 1),
    (17, 16, 1, 0, 1, 2),
    (129, 77, 1, 1, 1, 3),     # 5/3 inverse reads H with the D stride (odd width)
    (100, 60, 1, 31, 0, 4),
    (80, 64, 1, 20, 0, 5),
    (64, 64, 1, 9, 2, 6),      # haar, even at every level
    (96, 80, 3, 5, 0, 7),
    (48, 40, 3, 0, 1, 8),
    (121, 45, 1, 0, 1, 9),     # finest bands 61x23 / 60x23: 1x? edge cases
    (37, 37, 1, 0, 1, 10),     # finest D band 19x19: 1x? edges
    (101, 57, 1, 0, 1, 11),    # finest D 51x29 => ≡ 3 (mod 4) edges
]

BANDS = [  # (w, h, levels, lc, trans, q)
    (64, 48, 5, 1, 0, 9),
    (33, 47, 5, 1, 1, 0),
    (129, 77, 5, 1, 0, 5),
]


def sha(b):
    return hashlib.sha256(b).hexdigest()


def name_of(w, h, c, q, t, f):
    return "%s%dx%d_q%d_t%d_f%d" % ("rgb" if c == 3 else "g", w, h, q, t, f)


def main():
    ref = O.ref()
    if ref is None:
        raise SystemExit("oracle/_ref/libricref.so missing: run `make -C oracle` with /root/reference present")
    out = {"source": "reference library (oracle/_ref) in the build container", "small": [], "bands": [],
           "large": []}
    for (w, h, c, q, t, f) in SMALL:
        pix = O.synth(w, h, c, f)
        ric = ref.encode_ric(pix, q, t)
        nm = name_of(w, h, c, q, t, f)
        open(os.path.join(HERE, nm + ".ric"), "wb").write(ric)
        dec, planes = ref.decode_ric(ric)
        out["small"].append({"name": nm, "w": w, "h": h, "channels": c, "q": q, "trans": t, "frame": f,
                             "ric_bytes": len(ric), "ric_sha256": sha(ric), "decoded_sha256": sha(dec.tobytes()),
                             "planes_sha256": sha(planes.astype("<i2").tobytes())})
    for (w, h, L, lc, t, q) in BANDS:
        pl = O.gray_plane(O.synth(w, h, 1, 0)[0], q)
        Q = O.quants(q + 20) if q else 0
        lam = O.quants(q + 13) if q else 0
        # stage 0: after Transform, 1: after buildTree + LL TSUQ, 2: after the
        # whole CodeBand; 3: the closed loop CodeBand -> TSUQi -> TransformI
        # (src/lib/rududucodec.cpp:67-74), the reconstructed plane
        for stage in (0, 1, 2, 3):
            if stage == 3:
                flat = ref.closed_loop(pl, L, lc, t, Q, lam, Q or 1)[0].ravel().astype(np.int32)
            else:
                b = ref.bands(pl, L, lc, t, stage, Q, lam)
                flat = np.concatenate([x.ravel() for x in b]).astype(np.int32)
            nm = "bands_%dx%d_L%d_lc%d_t%d_q%d_s%d" % (w, h, L, lc, t, q, stage)
            np.save(os.path.join(HERE, nm + ".npy"), flat)
            out["bands"].append({"name": nm, "w": w, "h": h, "levels": L, "lc": lc, "trans": t, "q": q,
                                 "quant": Q, "lambda": lam, "stage": stage})
    # full-size configs (sha256 only)
    big = []
    img = O.synth(512, 512, 1)[0]
    pl = (img.astype(np.int32) - 128).astype(np.int16)
    buf = ref.encode_planes(pl[None], 3, -1, 1, [0], [0])
    big.append({"name": "C1_512x512_lossless_53_L3_lc-1", "kind": "planes", "w": 512, "h": 512, "levels": 3,
                "lc": -1, "trans": 1, "q": 0, "stream_bytes": len(buf), "stream_sha256": sha(buf)})
    for (nm, w, h, c, q, t, f) in [("C2_4096x4096_q9", 4096, 4096, 1, 9, 0, 0),
                                   ("C5_frame1_4096x4096_q9", 4096, 4096, 1, 9, 0, 1),
                                   ("C3_7680x4320_q9", 7680, 4320, 1, 9, 0, 0),
                                   ("lossless53_1001x603", 1001, 603, 1, 0, 1, 0),
                                   ("C3rgb_7680x4320_q9", 7680, 4320, 3, 9, 0, 0)]:
        pix = O.synth(w, h, c, f)
        ric = ref.encode_ric(pix, q, t)
        dec, _ = ref.decode_ric(ric)
        big.append({"name": nm, "kind": "ric", "w": w, "h": h, "channels": c, "q": q, "trans": t, "frame": f,
                    "ric_bytes": len(ric), "ric_sha256": sha(ric), "decoded_sha256": sha(dec.tobytes())})
    rgb = O.synth(7680, 4320, 3, 0)
    for ty in range(2):
        for tx in range(2):
            tile = np.ascontiguousarray(rgb[:, 2160 * ty:2160 * (ty + 1), 3840 * tx:3840 * (tx + 1)])
            ric = ref.encode_ric(tile, 9, 0)
            dec, _ = ref.decode_ric(ric)
            big.append({"name": "C4_tile_%d_%d" % (tx, ty), "kind": "tile", "tx": tx, "ty": ty, "w": 3840,
                        "h": 2160, "channels": 3, "q": 9, "trans": 0, "ric_bytes": len(ric), "ric_sha256": sha(ric),
                        "decoded_sha256": sha(dec.tobytes())})
    out["large"] = big
    json.dump(out, open(os.path.join(HERE, "golden.json"), "w"), indent=1)
    print("wrote", len(out["small"]), "small,", len(out["bands"]), "band dumps,", len(big), "large")


if __name__ == "__main__":
    main()
