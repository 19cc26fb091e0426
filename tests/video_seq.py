"""Synthetic video sequences for the video codec's parity tests, and the
binding of oracle/_ref/ricvid_ref (TEST INFRASTRUCTURE: the reference video
codec's classes compiled from /root/reference/src/lib, oracle/ref_video.cpp).

A sequence pans over a larger synthetic RGB image (SURVEY.md §8(d) generator)
by (dx, dy) pixels per frame, so the motion search has real motion to find;
frames are in CImage::inputSGI's layout (src/lib/image.cpp:96-123): planes R,
G, B, bottom row first."""
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF_BIN = os.path.join(REPO, "oracle", "_ref", "ricvid_ref")
BORDER = 15


def sequence(w, h, n, seed=0, dx=3, dy=2, margin=64):
    import ric_amd
    base = ric_amd.synth(w + margin, h + margin, 3, seed)
    out = np.empty((n, 3, h, w), np.uint8)
    for k in range(n):
        x0, y0 = (dx * k) % margin, (dy * k) % margin
        out[k] = base[:, y0:y0 + h, x0:x0 + w][:, ::-1, :]
    return out


def parse(blob, w, h, n):
    """ricvid_ref's output: per frame dict(size, stream, enc, dsize, dec, mv, bordered, yv12)"""
    frames, o = [], 0
    npl = 3 * w * h
    nb = 3 * (h + 2 * BORDER) * (w + 2 * BORDER)
    nmv = (w >> 3) * (h >> 3)
    for _ in range(n):
        size = int(np.frombuffer(blob, np.uint32, 1, o)[0]); o += 4
        stream = blob[o:o + size + 2]; o += size + 2
        enc = np.frombuffer(blob, np.int16, npl, o).reshape(3, h, w); o += 2 * npl
        dsize = int(np.frombuffer(blob, np.uint32, 1, o)[0]); o += 4
        dec = np.frombuffer(blob, np.int16, npl, o).reshape(3, h, w); o += 2 * npl
        mv = np.frombuffer(blob, np.uint32, nmv, o).reshape(h >> 3, w >> 3); o += 4 * nmv
        bord = np.frombuffer(blob, np.int16, nb, o).reshape(3, h + 2 * BORDER, w + 2 * BORDER); o += 2 * nb
        yv12 = blob[o:o + w * h * 3 // 2]; o += w * h * 3 // 2
        frames.append(dict(size=size, stream=stream, enc=enc, dsize=dsize, dec=dec, mv=mv, bordered=bord, yv12=yv12))
    assert o == len(blob), (o, len(blob))
    return frames


def ref_run(seq, q, tmpdir):
    """the reference video codec (encoder then decoder) on a sequence"""
    n, _, h, w = seq.shape
    src = os.path.join(str(tmpdir), "seq_%dx%d.rgb" % (w, h))
    dst = os.path.join(str(tmpdir), "ref_%dx%d_q%d.bin" % (w, h, q))
    np.ascontiguousarray(seq).tofile(src)
    subprocess.run([REF_BIN, str(w), str(h), str(q), str(n), src, dst], check=True, timeout=300)
    return parse(open(dst, "rb").read(), w, h, n)
