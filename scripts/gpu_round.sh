#!/bin/bash
# gpu_round.sh TAG -- the round's GPU evidence in one gpurun call:
# GPU parity tests, the contract bench line, then a rocprofv3 kernel-trace of
# a short bench.  Every GPU step has its own time limit; the first failure
# ends the script.
set -e -o pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
timeout -k 10 300 python3 -u bench.py > "$OUT/${TAG}_bench.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${TAG}_kt" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --steps 2 > "$OUT/${TAG}_kt.log" 2>&1
echo "round $TAG done"
