#!/bin/bash
# sweep_batch.sh TAG -- kbench_batch.py under tuning-knob variants (each its
# own process: the knobs are read once); one JSON line per variant in
# gpurun_out/TAG_sweep.jsonl.  Stops at the first run that does not exit 0.
TAG=${1:-sw}
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
: > "$OUT/${TAG}_sweep.jsonl"
VARS=${VARIANTS:-"NONE=1"}
for v in $VARS; do
  for s in ${SLOTS:-16}; do
    env $(echo "$v" | tr ',' ' ') timeout -k 10 120 python3 "$R/scripts/kbench_batch.py" --slots "$s" --iters ${ITERS:-10} \
        --tag "$v" >> "$OUT/${TAG}_sweep.jsonl" 2> "$OUT/${TAG}_sweep.err"
    rc=$?
    echo "$v slots=$s rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/${TAG}_sweep.err"; exit $rc; fi
  done
done
cat "$OUT/${TAG}_sweep.jsonl"
