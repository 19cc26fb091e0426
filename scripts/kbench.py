#!/usr/bin/env python3
"""kbench.py -- uncontended GPU stage timings on one 8K frame (single thread).

  python scripts/kbench.py [--iters N] [--width W --height H] [--codec]

Times the device stages in isolation with the library's HIP-event stage
timers: the fused forward DWT + quantiser + records (ric_transform_quantize;
"fwd_l0" = the level-0 kernel, "fwd" = the whole device encode, "quant" =
nothing unless RIC_NOFUSE=1 splits it off), then, with --codec, one full encode+decode per iteration on a
single codec (stage breakdown incl. the host coder).  Used for kernel tuning
and under rocprofv3; bench.py is the contract benchmark.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "rududu-image-codec_amd"))


def wgtrace_summary(ric_amd, path):
    """Per-workgroup timeline of the last traced level-0 launch: dispatch ramp,
    durations, producer SIMD placement; raw records go to `path`."""
    REC = 168
    n = 8192 * REC
    buf = np.zeros(n, np.uint64)
    got = ric_amd.lib().ric_diag_wgtrace(0, buf.ctypes.data, n)
    r = buf[:max(got, 0)].reshape(-1, REC)
    r = r[r[:, 0] != 0]
    if not len(r):
        return None
    t0 = r[:, 0].min()
    start = (r[:, 0] - t0) * 10.0 / 1e3            # us (100 MHz realtime)
    end = (r[:, 2:6].max(axis=1) - t0) * 10.0 / 1e3
    prod_end = np.zeros(len(r))
    hw = (r[:, 6] >> np.uint64(32)).astype(np.int64)
    clk = (r[:, 6] & np.uint64(0xFFFFFFFF)).astype(np.int64) - (r[:, 1] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    clk %= 1 << 32
    dur = end - start
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    xcc = (r[:, 7] >> np.uint64(32)).astype(np.int64) & 7
    key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    per_cu = {}
    for k, s_ in zip(key, simd):
        per_cu.setdefault(int(k), []).append(int(s_))
    same = sum(1 for v in per_cu.values() if len(v) != len(set(v)))
    ghz = np.median(clk / np.maximum(dur, 1e-3) / 1e3)
    np.save(path + ".npy", r)
    summ = {"wgs": int(len(r)), "span_us": round(float(end.max()), 2),
            "start_us_pct": [round(float(np.percentile(start, p)), 2) for p in (0, 10, 50, 90, 100)],
            "dur_us_pct": [round(float(np.percentile(dur, p)), 2) for p in (0, 10, 50, 90, 100)],
            "end_us_pct": [round(float(np.percentile(end, p)), 2) for p in (0, 10, 50, 90, 100)],
            "cus": len(per_cu), "wgs_per_cu_max": max(len(v) for v in per_cu.values()),
            "cus_with_shared_producer_simd": same, "shader_ghz_median": round(float(ghz), 3)}
    import json as _j
    with open(path, "w") as f:
        _j.dump(summ, f, indent=1)
    return summ


def gentrace_summary(ric_amd):
    """Phase stamps of the last traced k_fwdq_gen launch (RIC_LVL_TRACE=level):
    median / max microseconds from each workgroup's start to the end of its
    lifting, table staging, barrier, block phase and LL TSUQ."""
    REC = 168
    n = 8192 * REC
    buf = np.zeros(n, np.uint64)
    got = ric_amd.lib().ric_diag_wgtrace(0, buf.ctypes.data, n)
    r = buf[:max(got, 0)].reshape(-1, REC)[:, :9].astype(np.float64)
    r = r[r[:, 0] != 0]
    if not len(r):
        return None
    t0 = r[:, 0].min()
    out = {"wgs": int(len(r)), "start_us": [round(float(np.percentile((r[:, 0] - t0) / 100.0, p)), 2) for p in (50, 100)]}
    names = ["lift", "stage", "barrier", "blocks_w0", "blocks_w1", "blocks_w2", "blocks_w3", "ll"]
    for i, nm in enumerate(names, start=1):
        v = r[:, i]
        ok = v != 0
        if ok.any():
            d = (v[ok] - r[ok, 0]) / 100.0
            out[nm] = [round(float(np.median(d)), 2), round(float(d.max()), 2)]
    ends = r[:, 1:9].max(axis=1)
    out["span_us"] = round(float((ends.max() - t0) / 100.0), 2)
    return out


def pc2trace_summary(ric_amd):
    """Stamps of the last traced k_fwdq_pc2<true> launch (RIC_LVL_TRACE=1 or 2):
    medians over workgroups, microseconds from the workgroup's start."""
    REC = 168
    n = 8192 * REC
    buf = np.zeros(n, np.uint64)
    got = ric_amd.lib().ric_diag_wgtrace(0, buf.ctypes.data, n)
    r = buf[:max(got, 0)].reshape(-1, REC).astype(np.float64)
    r = r[r[:, 0] != 0]
    if not len(r):
        return None
    t0 = r[:, 0].min()
    rel = lambda c: (c - r[:, 0]) / 100.0
    med = lambda v: round(float(np.median(v)), 2)
    out = {"wgs": int(len(r)), "start_us": [med((r[:, 0] - t0) / 100.0), round(float((r[:, 0].max() - t0) / 100.0), 2)],
           "producers_done": [med(rel(r[:, 1])), med(rel(r[:, 2]))],
           "consumers_staged": [med(rel(r[:, 3 + b])) for b in range(3)],
           "consumers_done": [med(rel(r[:, 6 + b])) for b in range(3)],
           "span_us": round(float((r[:, 1:9].max() - t0) / 100.0), 2)}
    for b in range(3):
        rows = []
        for j in range(20):
            tk, fn = r[:, 16 + 20 * b + j], r[:, 96 + 20 * b + j]
            ok = (tk != 0) & (fn != 0)
            if not ok.any():
                break
            rows.append([med((tk[ok] - r[ok, 0]) / 100.0), med((fn[ok] - r[ok, 0]) / 100.0)])
        out["rows_b%d" % b] = rows
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--width", type=int, default=7680)
    ap.add_argument("--height", type=int, default=4320)
    ap.add_argument("--codec", action="store_true")
    ap.add_argument("--wgtrace", default="", help="write the level-0 workgroup trace summary (needs RIC_FQ_PC bit 128) to this json")
    ap.add_argument("--gentrace", action="store_true", help="stamp summary of the level named by RIC_LVL_TRACE")
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    import ric_amd
    W, H = a.width, a.height
    pix = ric_amd.synth(W, H, 1, 0)
    img = torch.from_numpy(((pix[0].astype(np.int16) - 128) << 4)).cuda()
    torch.cuda.synchronize()
    w = ric_amd.Wavelet2D(W, H, 5, 1)
    w.SetWeight(0)
    q, lam = ric_amd.quants(29), ric_amd.quants(22)
    out = {"config": "%dx%d gray 9/7 5 levels, Quant %d lambda %d" % (W, H, q, lam)}
    for i in range(a.warmup + a.iters):
        if i == a.warmup:
            w.prof_enable(True)
        w.TransformQuantize(img, W, 0, q, lam, on_device=True)
        w.prof_read()
    st = w.prof_read()
    out["wavelet_ms"] = {k: round(v[0] / v[1], 4) for k, v in st.items() if v[1]}
    fwd0 = out["wavelet_ms"].get("fwd_l0")
    if fwd0:
        out["fwd_l0_GBps"] = round(4.0 * W * H / (fwd0 * 1e-3) / 1e9, 1)
    enc = out["wavelet_ms"].get("fwd", 0) + out["wavelet_ms"].get("quant", 0)
    if enc:
        out["wavelet_encode_GBps"] = round(9.851 * W * H / (enc * 1e-3) / 1e9, 1)
    if a.wgtrace:
        out["wgtrace"] = wgtrace_summary(ric_amd, a.wgtrace)
    if a.gentrace:
        lvl = int(os.environ.get("RIC_LVL_TRACE", "-1"))
        out["lvltrace"] = pc2trace_summary(ric_amd) if lvl in (1, 2) else gentrace_summary(ric_amd)
    if a.codec:
        c = ric_amd.Codec(W, H, 1)
        dpix = torch.from_numpy(pix).cuda()
        dout = torch.empty_like(dpix)
        for i in range(a.warmup + a.iters):
            if i == a.warmup:
                c.prof_enable(True)
                t0 = time.perf_counter()
            ric = c.compress(dpix, q=9, trans=0, on_device=True)
            c.decompress(ric, pix_out=dout)
        dt = (time.perf_counter() - t0) / a.iters
        st = c.prof_read()
        out["codec_ms"] = {k: round(v[0] / v[1], 4) for k, v in st.items() if v[1]}
        out["codec_frame_ms"] = round(dt * 1e3, 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
