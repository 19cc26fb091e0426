#!/bin/bash
# gpu_check.sh TAG [quick] -- GPU parity tests (default path, then every 9/7
# level through the generic fused kernel), then kernel timings under
# rocprofv3 and a few tuning-knob variants.  Run via gpurun.  quick: skip
# the tests.
set -e -o pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
if [ "$2" != "quick" ]; then
  timeout -k 10 400 python3 -m pytest tests -m gpu -x -q > "$OUT/${TAG}_t.log" 2>&1
  RIC_DWT_NOFAST=1 timeout -k 10 300 python3 -m pytest tests/test_gpu_golden.py tests/test_gpu_parity.py -m gpu -x -q > "$OUT/${TAG}_tnf.log" 2>&1
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${TAG}_kt" -o run -- \
    python3 "$R/scripts/kbench.py" --iters 20 --codec > "$OUT/${TAG}_kb.log" 2>&1
for v in ${VARIANTS:-"RIC_FQ_GEN_BELOW=4096" "RIC_NOFUSE=1"}; do
  n=${v//=/_}
  env "$v" timeout -k 10 200 python3 "$R/scripts/kbench.py" --iters 20 > "$OUT/${TAG}_kb_$n.log" 2>&1
done
echo "check $TAG done"
