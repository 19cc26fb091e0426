import sys, numpy as np
sys.path.insert(0,'rududu-image-codec_amd'); sys.path.insert(0,'.')
import torch, ric_amd
from oracle import oracle as O
port = O.port()
w, h, q, t = 1001, 603, 0, 1
for n in (1, 3):
    rics = [port.encode_ric(ric_amd.synth(w, h, 1, 90 + i), q, t) for i in range(n)]
    istride = (max(len(r) for r in rics) + 4095) // 4096 * 4096
    buf = np.zeros(n * istride, np.uint8)
    for i, r in enumerate(rics):
        buf[i * istride:i * istride + len(r)] = np.frombuffer(r, np.uint8)
    src = torch.from_numpy(buf).cuda()
    outs = [torch.zeros((1, h, w), dtype=torch.uint8, device="cuda") for _ in rics]
    b = ric_amd.Batch(w, h, 1, slots=n, threads=1)
    rc = b.decompress_gpu(src, istride, [len(r) for r in rics], outs)
    hb = b.decompress(rics)
    for i in range(n):
        o = port.decode_ric(rics[i])[0].reshape(h, w)
        g = outs[i].cpu().numpy().reshape(h, w)
        print("n=%d frame %d rc %d gpu==oracle %s host-batch==oracle %s ndiff %d" % (n, i, rc, np.array_equal(g, o), np.array_equal(hb[i].reshape(h, w), o), int((g != o).sum())))
