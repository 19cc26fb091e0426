#!/bin/bash
# pmc_sweep.sh TAG "COUNTERS1" "COUNTERS2" ... -- one rocprofv3 --pmc pass per
# argument over scripts/kbench.py (run on the GPU box); stops at the first failure.
set -e -o pipefail
TAG=$1; shift
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
k=0
for ctrs in "$@"; do
  k=$((k+1))
  timeout -k 10 200 rocprofv3 --pmc $ctrs -f csv -d "$R/gpurun_out/${TAG}_p$k" -o run -- \
      python3 "$R/scripts/kbench.py" --iters 5 --warmup 1 > "$R/gpurun_out/${TAG}_p$k.log" 2>&1
done
echo pmc done
