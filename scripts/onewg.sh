#!/bin/bash
# onewg.sh TAG -- latency experiments on the producer-consumer level kernel
# (timing only, results invalid).  RIC_FQ_PC bits: 2 = consumers idle,
# 8 = no input loads, 16 = no LDS/L stores; RIC_FQ_ONEWG=1 = one workgroup.
set -e -o pipefail
TAG=$1
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in ${ONEWG_VARIANTS:-"RIC_FQ_ONEWG=1 RIC_FQ_PC=2" "RIC_FQ_ONEWG=1 RIC_FQ_PC=10" "RIC_FQ_ONEWG=1 RIC_FQ_PC=26" "RIC_FQ_PC=2" "RIC_FQ_PC=10" "RIC_FQ_PC=26" "RIC_FQ_PC=1"}; do
  n=$(echo $v | tr ' =' '__')
  env $v timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/${TAG}_$n" -o run -- \
      python3 "$R/scripts/kbench.py" --iters 10 > "$R/gpurun_out/${TAG}_$n.log" 2>&1
done
echo onewg done
