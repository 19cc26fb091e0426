#!/bin/bash
# r2_gc_profile.sh TAG -- rocprofv3 evidence for the default bench (GPU stream
# coder at C3): kernel trace + stats of bench.py itself (1 timed step), then
# the SQ instruction counters of the stream coder kernels at 1080p (one pass).
set -o pipefail
TAG=${1:-r2gc}
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {   # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -1 "$OUT/${TAG}_${name}.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
run bkt 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${TAG}_bkt" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline
run sq 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM \
    -f csv -d "$OUT/${TAG}_sq" -o run -- python3 "$R/scripts/gc_probe.py" --w 1920 --h 1080 --n 8 --reps 1 --check 1
echo "profile $TAG done"
