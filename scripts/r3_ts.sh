#!/bin/bash
# r3_ts.sh TAG -- the stream coder tests, then the default bench with every
# coder wave's start / end summarised per launch (RIC_GC_TSTAMP) and the step
# timeline (RIC_HYBRID_TRACE) on stderr.  The first failure ends the script.
set -e -o pipefail
TAG=$1
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
[ -n "$NOTEST" ] || timeout -k 10 300 python3 -u -m pytest tests/test_gpu_coder.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
RIC_GC_TSTAMP=1 RIC_GC_TSTAMP_FILE=$OUT/${TAG}_waves.txt RIC_HYBRID_TRACE=1 timeout -k 10 420 python3 -u bench.py --no-cpu-baseline --no-latency \
	> "$OUT/${TAG}_bench.log" 2> "$OUT/${TAG}_bench.err"
echo "ts $TAG done"
