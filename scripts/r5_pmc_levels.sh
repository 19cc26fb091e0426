#!/bin/bash
# r5_pmc_levels.sh TAG -- HBM bytes of every forward level kernel of the
# isolated 5-level encode (scripts/kbench_batch.py, 16 C3 frames per launch):
# rocprofv3 --pmc FETCH_SIZE and WRITE_SIZE in separate passes (one TCC
# counter group each, MI355X_MICROARCH.md HBM section), then the kernel trace
# of the same command; via gpurun.  Summarised by scripts/pmc_levels.py.
set -e -o pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $C -f csv -d "$OUT/${TAG}_pmc_${C}" -o run -- \
      python3 "$R/scripts/kbench_batch.py" --iters 3 > "$OUT/${TAG}_pmc_${C}.log" 2>&1
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${TAG}_kt" -o run -- \
    python3 "$R/scripts/kbench_batch.py" --iters 10 > "$OUT/${TAG}_kt.log" 2>&1
echo "pmc levels $TAG done"
