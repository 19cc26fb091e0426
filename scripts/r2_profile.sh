#!/bin/bash
# r2_profile.sh TAG -- rocprofv3 evidence for the batched path (run via gpurun):
#   TAG_bkt   kernel trace + stats of bench.py itself (3 steps)
#   TAG_kkt   kernel trace + stats of the GPU stages alone (scripts/kbench_batch.py)
#   TAG_pmc_fetch / TAG_pmc_write   FETCH_SIZE and WRITE_SIZE, one counter per pass
# Each step has its own time limit; the script stops at the first failure.
set -o pipefail
TAG=${1:-r2p}
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {   # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "$OUT/${TAG}_${name}.log"
  [ $rc -eq 0 ] || exit $rc
}
run bkt 400 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${TAG}_bkt" -o run -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-split
run kkt 200 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${TAG}_kkt" -o run -- \
    python3 "$R/scripts/kbench_batch.py" --slots 16 --iters 10
run pmcf 200 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/${TAG}_pmc_fetch" -o run -- \
    python3 "$R/scripts/kbench_batch.py" --slots 16 --iters 2
run pmcw 200 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/${TAG}_pmc_write" -o run -- \
    python3 "$R/scripts/kbench_batch.py" --slots 16 --iters 2
echo "profile $TAG done"
