#!/bin/bash
# r3_ab_env.sh TAG VAR "V1 V2 ..." -- the stream coder tests (unless NOTEST),
# then the default bench once per value of the environment variable VAR,
# wave stamps (TSTAMP=1) and the step timeline on stderr.
set -e -o pipefail
TAG=$1; VAR=$2; VALS=$3
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
[ -n "$NOTEST" ] || timeout -k 10 300 python3 -u -m pytest tests/test_gpu_coder.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
for V in $VALS; do
	env "$VAR=$V" RIC_GC_TSTAMP=${TSTAMP:-0} RIC_GC_TSTAMP_FILE=$OUT/${TAG}_${V}_waves.txt RIC_HYBRID_TRACE=1 \
		timeout -k 10 420 python3 -u bench.py --no-cpu-baseline --no-latency $BENCH_ARGS \
		> "$OUT/${TAG}_${V}_bench.log" 2> "$OUT/${TAG}_${V}_bench.err"
done
echo "ab $TAG done"
