#!/bin/bash
# gpu_evidence.sh TAG -- the committed GPU evidence of a round, in one gpurun
# call: GPU parity tests, the contract bench line, rocprofv3 kernel trace of
# a short bench, and the FETCH_SIZE / WRITE_SIZE passes (separate runs) over
# scripts/kbench.py for the level-0 fused kernel's HBM traffic.
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
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/${TAG}_pmc_fetch" -o run -- \
    python3 "$R/scripts/kbench.py" --iters 3 --warmup 1 > "$OUT/${TAG}_pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/${TAG}_pmc_write" -o run -- \
    python3 "$R/scripts/kbench.py" --iters 3 --warmup 1 > "$OUT/${TAG}_pmc_write.log" 2>&1
echo "evidence $TAG done"
