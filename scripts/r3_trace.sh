#!/bin/bash
# r3_trace.sh TAG -- one warmup + one timed step of the default bench under
# rocprofv3 (kernel + memory-copy trace), the step timeline on stderr.
set -e -o pipefail
TAG=$1
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
RIC_HYBRID_TRACE=1 timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/${TAG}_prof" -o run --output-format csv -- \
	python3 -u "$OLDPWD/bench.py" --no-cpu-baseline --no-latency --no-verify --steps 1 --warmup 1 $BENCH_ARGS \
	> "$OUT/${TAG}_bench.log" 2> "$OUT/${TAG}_bench.err"
echo "trace $TAG done"
