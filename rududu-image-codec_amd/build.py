"""Build librududu_amd.so in-tree: HIP kernels with hipcc for gfx950, host
sources with g++ against the ROCm headers.  Usage: python build.py [-j N]."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "librududu_amd.so")
OBJ = os.path.join(HERE, "build")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("RIC_OFFLOAD_ARCH", "gfx950")

COMMON = ["-O3", "-std=c++17", "-fPIC", "-fwrapv", "-I" + os.path.join(REPO, "include"), "-I" + CSRC]
HOSTCXX = os.environ.get("RIC_HOST_CXX") or next(
    (c for c in (os.path.join(ROCM, "llvm", "bin", "clang++"),) if os.path.exists(c)), "g++")


def _sources():
    return sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def _headers_mtime():
    m = 0.0
    for d in (CSRC, os.path.join(REPO, "include")):
        for f in os.listdir(d):
            if f.endswith((".h", ".inc")):
                m = max(m, os.path.getmtime(os.path.join(d, f)))
    return m


def _compile(src, hdr_mtime):
    path = os.path.join(CSRC, src)
    obj = os.path.join(OBJ, src + ".o")
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(path), hdr_mtime):
        return obj
    if src.endswith(".hip"):
        cmd = [os.path.join(ROCM, "bin", "hipcc"), "--offload-arch=" + ARCH] + COMMON + ["-c", path, "-o", obj]
    else:
        # host sources (the serial coder): x86-64-v3 (AVX2/BMI2/LZCNT, present on the
        # GPU boxes' EPYC and this container's Xeon): encoder -7 %.  ROCm's clang
        # rather than g++ 11: the host coder 5-6 % faster on the box's EPYC 9575F
        # (scripts/hostbench, one C3 frame: encode 102.8 -> 97.6 ms, decode 120.3 -> 112.9).
        # Scheduled for the box's Zen 5 (-mtune only: the code still runs here;
        # decode -1 %).
        tune = ["-mtune=znver5"] if "clang" in os.path.basename(HOSTCXX) else []
        cmd = [HOSTCXX] + COMMON + ["-march=x86-64-v3", "-Wall"] + tune + [
            "-D__HIP_PLATFORM_AMD__", "-I" + os.path.join(ROCM, "include"), "-c", path, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("compile failed: %s\n%s" % (" ".join(cmd), r.stderr))
    return obj


def build(jobs=8, verbose=False):
    os.makedirs(OBJ, exist_ok=True)
    hdr = _headers_mtime()
    srcs = _sources()
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hdr), srcs))
    if os.path.exists(OUT) and os.path.getmtime(OUT) >= max(os.path.getmtime(o) for o in objs):
        _build_cli()
        return OUT
    cmd = [os.path.join(ROCM, "bin", "hipcc"), "--offload-arch=" + ARCH, "-shared", "-fPIC"] + objs + [
        "-L" + os.path.join(ROCM, "lib"), "-lrccl", "-Wl,-rpath," + os.path.join(ROCM, "lib"), "-o", OUT]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("link failed: %s\n%s" % (" ".join(cmd), r.stderr))
    _build_cli()
    if verbose:
        print("built", OUT)
    return OUT


def _build_cli():
    """tools/ric_cli.cpp -> ./ric (the src/ric/ric.cpp counterpart, rpath to the .so)."""
    src = os.path.join(HERE, "tools", "ric_cli.cpp")
    exe = os.path.join(HERE, "ric")
    deps = [src, OUT, os.path.join(REPO, "include", "rududu_gpu.hpp"), os.path.join(REPO, "include", "ric_gpu.h")]
    if os.path.exists(exe) and os.path.getmtime(exe) >= max(os.path.getmtime(d) for d in deps):
        return exe
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-I" + os.path.join(REPO, "include"), src, "-o", exe,
           "-L" + HERE, "-lrududu_amd", "-Wl,-rpath,$ORIGIN"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("cli build failed: %s\n%s" % (" ".join(cmd), r.stderr))
    return exe


if __name__ == "__main__":
    j = int(sys.argv[sys.argv.index("-j") + 1]) if "-j" in sys.argv else 8
    build(j, verbose=True)
