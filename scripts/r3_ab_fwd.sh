#!/bin/bash
# r3_ab_fwd.sh TAG -- the default bench with the step's forward levels ahead of
# the coder launches (RIC_FWD_AHEAD=1, the default) and without (0), both with
# the step timeline on stderr.  The first failure ends the script.
set -e -o pipefail
TAG=$1
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
for A in 1 0; do
	RIC_FWD_AHEAD=$A RIC_HYBRID_TRACE=1 timeout -k 10 420 python3 -u bench.py --no-cpu-baseline --no-latency \
		> "$OUT/${TAG}_a${A}_bench.log" 2> "$OUT/${TAG}_a${A}_bench.err"
done
echo "ab $TAG done"
