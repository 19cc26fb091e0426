#!/bin/bash
# gpu_pcs.sh TAG [probe args...] -- PC sampling (host trap) of the GPU stream
# coder over scripts/gc_probe.py, to find the coder's hot instructions (map the
# sampled code-object offsets onto `llvm-objdump -d` of the library's gfx950
# code object).  One GPU step, time-limited.
set -e -o pipefail
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$OUT/${TAG}_avail.txt" 2>&1 || true
timeout -k 10 400 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
    --pc-sampling-interval 256 -f csv -d "$OUT/${TAG}_pcs" -o run -- \
    python3 "$R/scripts/gc_probe.py" "$@" > "$OUT/${TAG}_pcs.log" 2>&1
echo "pcs $TAG done"
