#!/bin/bash
# s4_final.sh TAG -- end-of-session GPU evidence in one call: the GPU parity
# suite, the driver's bench command (--steps 20 --warmup 5), and a rocprofv3
# kernel trace of a short bench; each step under its own limit, stop at the
# first failure.
TAG=${1:-s4fin}
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
run() { local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/${TAG}_${name}.log" 2> "$OUT/${TAG}_${name}.err"; local rc=$?
  echo "$name rc=$rc"; tail -2 "$OUT/${TAG}_${name}.log" | cut -c1-400
  [ $rc -eq 0 ] || exit $rc; }
run tests 500 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
run bench 560 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp
run kt 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${TAG}_kt" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --steps 2 --warmup 2
echo "final $TAG done"
