#!/bin/bash
# r6_prio_ab.sh TAG MODES... -- coder tests under RIC_GC_PRIO=<first mode>,
# then one short bench per mode (wave end tiers from RIC_GC_TSTAMP).  Via gpurun.
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out
mkdir -p "$OUT"
RIC_GC_PRIO=$1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_coder.py -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "hybrid or roundtrip or large_sha" > "$OUT/${TAG}_tests.log" 2>&1
echo "tests ok"
for m in "$@"; do
  RIC_GC_PRIO=$m RIC_GC_TSTAMP=1 timeout -k 10 400 python3 -u bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-latency \
      --no-split > "$OUT/${TAG}_p$m.log" 2> "$OUT/${TAG}_p$m.err"
  echo "mode $m: $(grep -o '"value": [0-9.]*' $OUT/${TAG}_p$m.log) $(grep -o '"ms_per_launch": [0-9.]*' $OUT/${TAG}_p$m.log)"
done
