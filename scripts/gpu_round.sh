#!/bin/bash
# gpu_round.sh TAG [STEPS] -- one gpurun call's GPU evidence: the GPU parity
# tests, the driver's smoke(), the contract bench line, then a rocprofv3
# kernel-trace (--stats) of the default bench at this tree.  Every GPU step
# has its own time limit; the first failure ends the script.
set -e -o pipefail
TAG=$1
STEPS=${2:-3}
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/${TAG}_smoke.log" 2>&1
timeout -k 10 400 python3 -u bench.py --steps "$STEPS" > "$OUT/${TAG}_bench.log" 2> "$OUT/${TAG}_bench.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${TAG}_kt" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-latency --steps 1 > "$OUT/${TAG}_kt.log" 2> "$OUT/${TAG}_kt.err"
echo "round $TAG done"
