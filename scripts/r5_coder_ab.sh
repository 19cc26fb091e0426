#!/bin/bash
# r5_coder_ab.sh TAG LIB... -- the stream coder alone (one C3 serving step of
# 3072 GPU streams, no host frames) under each library build ("-" = the
# tree's), after a quick parity check of that build; via gpurun
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out
mkdir -p "$OUT"
for L in "$@"; do
  if [ "$L" = "-" ]; then unset RIC_AMD_LIB; n=tree; else export RIC_AMD_LIB=$(pwd)/$L; n=$(basename "$L" .so); fi
  timeout -k 10 200 python3 -u -m pytest tests/test_gpu_coder.py -m gpu -x -q --timeout 120 --timeout-method thread \
      -k "matches_oracle or large_sha" > "$OUT/${TAG}_${n}_t.log" 2>&1
  timeout -k 10 300 python3 -u bench.py --steps 1 --warmup 1 --n-host 0 --no-verify --no-cpu-baseline --no-latency \
      > "$OUT/${TAG}_${n}_b.log" 2> "$OUT/${TAG}_${n}_b.err"
done
echo "coder ab $TAG done"
