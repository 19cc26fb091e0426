#!/bin/bash
# dwt_sweep.sh TAG -- kernel-trace kbench under DWT tuning knobs (run on the GPU box)
set -e -o pipefail
TAG=$1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for cfg in ${CFGS:-"def" "RIC_DWT_NOFAST=1" "RIC_DWT_S=8" "RIC_DWT_S=16" "RIC_DWT_S=32" "RIC_DWT_S=64"}; do
  name=${cfg//=/_}
  if [ "$cfg" = "def" ]; then unset RIC_DWT_NOFAST RIC_DWT_S; else export "$cfg"; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/${TAG}_${name}_kt" -o run -- \
      python3 "$R/scripts/kbench.py" --iters 10 > "$R/gpurun_out/${TAG}_${name}.log" 2>&1
  unset RIC_DWT_NOFAST RIC_DWT_S
done
echo sweep done
