"""The serial .ric coder on the GPU (gcoder.hip: one wave per frame's stream)
against the oracle and the golden vectors: ric_batch_encode_gpu must write the
same .ric bytes as the reference's CompressImage."""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
G = json.load(open(os.path.join(HERE, "golden", "golden.json")))


def _gpu_encode(ric, frames, q, t):
    import torch
    h, w = frames[0].shape[-2:]
    dev = [torch.from_numpy(np.ascontiguousarray(f)).cuda() for f in frames]
    b = ric.Batch(w, h, 1, slots=len(frames), threads=1)
    ostride = (w * h * 2 + 65536 + 4095) // 4096 * 4096
    out = torch.zeros(len(frames) * ostride, dtype=torch.uint8, device="cuda")
    lens = b.compress_gpu(dev, out, ostride, q, t)
    host = out.cpu().numpy()
    return [host[i * ostride:i * ostride + n].tobytes() for i, n in enumerate(lens)]


@pytest.mark.parametrize("w,h,q,t", [(1024, 768, 9, 0), (640, 480, 0, 1), (328, 200, 20, 0), (257, 129, 9, 0),
                                     (128, 96, 9, 2), (1001, 603, 0, 1), (33, 47, 9, 0), (17, 16, 0, 1),
                                     (100, 60, 31, 0), (129, 77, 1, 1), (520, 392, 5, 0)])
def test_gpu_coder_matches_oracle(ric, port, w, h, q, t):
    frames = [ric.synth(w, h, 1, 60 + i) for i in range(3)]
    got = _gpu_encode(ric, frames, q, t)
    for f, r in zip(frames, got):
        assert r == port.encode_ric(f, q, t)


def test_gpu_coder_golden_small(ric):
    """Every small gray golden .ric of the reference, re-encoded on the GPU."""
    n = 0
    for e in G["small"]:
        if e["channels"] != 1:
            continue
        frame = ric.synth(e["w"], e["h"], 1, e["frame"])
        got = _gpu_encode(ric, [frame], e["q"], e["trans"])[0]
        assert got == open(os.path.join(HERE, "golden", e["name"] + ".ric"), "rb").read(), e["name"]
        n += 1
    assert n >= 8


@pytest.mark.parametrize("name", ["C3_7680x4320_q9", "C2_4096x4096_q9"])
def test_gpu_coder_large_sha(ric, name):
    """Full-size frames: the reference's own SHA-256 of the .ric file."""
    e = [x for x in G["large"] if x["name"] == name][0]
    w, h = e["w"], e["h"]
    frame = ric.synth(w, h, 1, e["frame"])
    got = _gpu_encode(ric, [frame], e["q"], e["trans"])[0]
    assert hashlib.sha256(got).hexdigest() == e["ric_sha256"]
