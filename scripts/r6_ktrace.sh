#!/bin/bash
# r6_ktrace.sh TAG [BENCH_ARGS...] -- the bench under rocprofv3 --kernel-trace
# --stats (via gpurun); the summary and a step timeline (scripts/step_timeline.py)
# are what to keep.  The raw trace stays in gpurun_out (compressed).
set -e -o pipefail
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${TAG}_kt" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-latency --no-split "$@" > "$OUT/${TAG}_kt.log" 2>&1
cd "$R"
KT=$(find "$OUT/${TAG}_kt" -name "*kernel_trace.csv" | head -1)
python3 scripts/step_timeline.py "$KT" > "$OUT/${TAG}_timeline.txt"
gzip -f "$KT"
echo "ktrace $TAG done"
