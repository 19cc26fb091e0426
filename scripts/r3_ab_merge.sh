#!/bin/bash
# r3_ab_merge.sh TAG -- the default bench with both coder halves as one launch
# (RIC_GC_MERGE=1, the default) and as two (0), step timeline on stderr.
set -e -o pipefail
TAG=$1
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
for A in ${ORDER:-1 0}; do
	RIC_GC_MERGE=$A RIC_HYBRID_TRACE=1 timeout -k 10 420 python3 -u bench.py --no-cpu-baseline --no-latency $BENCH_ARGS \
		> "$OUT/${TAG}_m${A}_bench.log" 2> "$OUT/${TAG}_m${A}_bench.err"
done
echo "ab $TAG done"
