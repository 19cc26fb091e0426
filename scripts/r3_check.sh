#!/bin/bash
# r3_check.sh TAG [pytest targets...] -- GPU tests of the given files, then the
# default bench line.  Each GPU step has its own time limit; the first failure
# ends the script.
set -e -o pipefail
TAG=$1; shift
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
timeout -k 10 600 python3 -u bench.py > "$OUT/${TAG}_bench.log" 2> "$OUT/${TAG}_bench.err"
echo "check $TAG done"
