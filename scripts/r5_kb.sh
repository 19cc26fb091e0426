#!/bin/bash
# r5_kb.sh TAG -- isolated batch kernel timings (scripts/kbench_batch.py) under
# knob settings, on the GPU box (via gpurun).  KB_VARIANTS: settings separated
# by '|', the variables of one setting by ':'
set -e -o pipefail
TAG=$1
OUT=gpurun_out
mkdir -p "$OUT"
IFS='|' read -r -a VS <<< "${KB_VARIANTS:-RIC_PIX8=1|RIC_PIX8=0}"
for v in "${VS[@]}"; do
  env ${v//:/ } timeout -k 10 120 python3 -u scripts/kbench_batch.py --iters 10 --slots "${KB_SLOTS:-16}" --tag "$v" >> "$OUT/${TAG}_kb.log" 2>&1
done
echo "kb $TAG done"
