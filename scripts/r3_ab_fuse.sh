#!/bin/bash
# r3_ab_fuse.sh TAG -- the stream coder tests, then the default bench with the
# merged coder launch as one encode+decode kernel (RIC_GC_FUSE=1, default) and
# as two kernels (0); timeline and wave stamps on stderr.
set -e -o pipefail
TAG=$1
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
[ -n "$NOTEST" ] || timeout -k 10 300 python3 -u -m pytest tests/test_gpu_coder.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
for A in ${ORDER:-1 0}; do
	RIC_GC_FUSE=$A RIC_GC_TSTAMP=${TSTAMP:-1} RIC_HYBRID_TRACE=${HTRACE:-1} timeout -k 10 420 python3 -u bench.py --no-cpu-baseline --no-latency $BENCH_ARGS \
		> "$OUT/${TAG}_f${A}_bench.log" 2> "$OUT/${TAG}_f${A}_bench.err"
done
echo "ab $TAG done"
