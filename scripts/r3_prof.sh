#!/bin/bash
# r3_prof.sh TAG -- (1) the default bench under rocprofv3 --kernel-trace
# --stats (kernel summary kept, the per-dispatch trace dropped: too large to
# bring back); (2) the default bench again with every coder wave's start / end
# / placement recorded (RIC_GC_TSTAMP_FILE).  The first failure ends the script.
set -e -o pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${TAG}_kt" -o run -- \
	python3 -u "$R/bench.py" --no-cpu-baseline > "$OUT/${TAG}_kt.log" 2> "$OUT/${TAG}_kt.err"
find "$OUT/${TAG}_kt" -name "*_kernel_trace.csv" -delete
cd "$R"
RIC_GC_TSTAMP=1 RIC_GC_TSTAMP_FILE=$OUT/${TAG}_waves.txt RIC_HYBRID_TRACE=1 timeout -k 10 420 python3 -u bench.py --no-cpu-baseline --no-latency \
	> "$OUT/${TAG}_ts.log" 2> "$OUT/${TAG}_ts.err"
echo "prof $TAG done"
