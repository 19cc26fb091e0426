"""Debug the video codec against the reference frame by frame: the OBMC
prediction and the wavelet closed loop on the reference's own residual
planes.  python scripts/dbg/video_debug.py W H Q N SEED FRAME"""
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "rududu-image-codec_amd"), REPO]
import torch  # noqa: E402
torch.cuda.init()
import ric_amd  # noqa: E402
import video_seq  # noqa: E402
from oracle import oracle as O  # noqa: E402


def vq(idx):
    Q = [32768, 37641, 43238, 49667, 57052]
    if idx == 0:
        return 0
    idx -= 1
    r = 10 - idx // 5
    return int(np.int16((Q[idx % 5] + (1 << (r - 1))) >> r))


def diff(a, b):
    d = np.argwhere(a != b)
    return "equal" if d.size == 0 else "%d differ, first %s: %d vs %d" % (len(d), tuple(d[0]), a[tuple(d[0])], b[tuple(d[0])])


w, h, q, n, seed, F = (int(x) for x in sys.argv[1:7])
td = tempfile.mkdtemp()
seq = video_seq.sequence(w, h, n, seed)
seq.tofile(os.path.join(td, "s.rgb"))
env = dict(os.environ, RICVID_DUMP=td)
subprocess.run([video_seq.REF_BIN, str(w), str(h), str(q), str(n), os.path.join(td, "s.rgb"), os.path.join(td, "o.bin")],
               env=env, check=True)
want = video_seq.parse(open(os.path.join(td, "o.bin"), "rb").read(), w, h, n)
enc = ric_amd.VideoCodec(True, w, h)
enc.quant = q
B = 15
for k in range(F + 1):
    s = enc.encode(seq[k])
    print("frame %d: mv %s | enc %s | stream %s" % (k, diff(enc.motion(), want[k]["mv"]),
                                                    diff(enc.output(True), want[k]["bordered"]),
                                                    "equal" if s == want[k]["stream"] else "DIFF"))
    pf = os.path.join(td, "pred_f%d.i16" % k)
    if os.path.exists(pf):
        rp = np.fromfile(pf, np.int16).reshape(3, h + 30, w + 30)
        gp = enc.prediction()
        print("   pred interior %s" % diff(gp[:, B:B + h, B:B + w], rp[:, B:B + h, B:B + w]))
# the closed loop on the reference's residual planes of frame F
res = np.fromfile(os.path.join(td, "res_f%d.i16" % F), np.int16).reshape(3, h + 30, w + 30)[:, B:B + h, B:B + w]
ref = O.ref()
for c in range(3):
    pl = np.ascontiguousarray(res[c])
    exp_plane, exp_bands = ref.closed_loop(pl, 3, 0, 0, vq(q + 20), vq(q + 12), vq(q + 20))
    W = ric_amd.Wavelet2D(w, h, 3, 0)
    W.SetWeight(0)
    W.Transform(pl, w, 0)
    buf = np.zeros(w * h * 8 + 4096, np.uint8)
    m = ric_amd.MuxCodec(buf, first_word=0)
    W.CodeBand(m, vq(q + 20), vq(q + 12))
    m.endCoding()
    W.TSUQi(vq(q + 20))
    gb = W.bands()
    bd = [i for i, (a, b) in enumerate(zip(gb, exp_bands)) if not np.array_equal(a, b)]
    out = np.zeros((h, w), np.int16)
    W.TransformI(out, w, 0)
    print("closed loop plane %d: bands differing %s; plane %s" % (c, bd, diff(out, exp_plane)))
    for i in bd[:3]:
        print("   band %d: %s" % (i, diff(gb[i], exp_bands[i])))
    # band dumps after Transform (stage 0) and after buildTree (1)
    for stage in (0, 1, 2):
        eb = ref.bands(pl, 3, 0, 0, stage, vq(q + 20), vq(q + 12))
        W2 = ric_amd.Wavelet2D(w, h, 3, 0)
        W2.SetWeight(0)
        W2.Transform(pl, w, 0)
        if stage == 1:
            W2.Quantize(vq(q + 20), vq(q + 12))
        elif stage == 2:
            m2 = ric_amd.MuxCodec(np.zeros(w * h * 8 + 4096, np.uint8), first_word=0)
            W2.CodeBand(m2, vq(q + 20), vq(q + 12))
        g2 = W2.bands()
        print("   stage %d differing bands %s" % (stage, [i for i, (a, b) in enumerate(zip(g2, eb)) if not np.array_equal(a, b)]))
