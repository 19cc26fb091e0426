#!/bin/bash
# gc_check.sh TAG -- the GPU stream coder on the GPU box: its parity tests,
# then encode/decode probes (1080p and C3), each step under its own limit;
# stops at the first step that does not end cleanly.
TAG=${1:-gc}
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
step() {   # name limit cmd...
  local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -3 "$OUT/${TAG}_${name}.log" | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step tests 500 python3 -u -m pytest tests/test_gpu_coder.py -m gpu -x -q --timeout 240 --timeout-method thread
step p1080 200 python3 -u scripts/gc_probe.py --w 1920 --h 1080 --n 64 --reps 1 --check 2
step pc3 300 python3 -u scripts/gc_probe.py --w 7680 --h 4320 --n 16 --reps 1 --check 2
echo "gc_check $TAG done"
