#!/bin/bash
# r3_etab.sh TAG -- GPU coder + batch tests, the decoder A/B (enum table on /
# off, 1080p x 1024 streams), then the default bench.
set -e -o pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_coder.py tests/test_gpu_batch.py -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
RIC_GC_ETAB=0 timeout -k 10 200 python3 -u scripts/gc_probe.py --w 1920 --h 1080 --n 1024 --reps 2 --check 1 > "$OUT/${TAG}_probe_e0.log" 2>&1
RIC_GC_ETAB=1 timeout -k 10 200 python3 -u scripts/gc_probe.py --w 1920 --h 1080 --n 1024 --reps 2 --check 1 > "$OUT/${TAG}_probe_e1.log" 2>&1
timeout -k 10 900 python3 -u bench.py > "$OUT/${TAG}_bench.log" 2> "$OUT/${TAG}_bench.err"
echo "etab $TAG done"
