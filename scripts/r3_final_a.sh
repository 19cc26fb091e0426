#!/bin/bash
# r3_final_a.sh TAG -- the whole GPU suite, then the stream coder's SQ / GRBM
# counters at 2816 1080p streams in flight (scripts/r3_sq2816.sh).
set -e -o pipefail
TAG=$1
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/${TAG}_all.log" 2>&1
bash scripts/r3_sq2816.sh "$TAG"
echo "final_a $TAG done"
