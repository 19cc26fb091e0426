#!/bin/bash
# variants.sh TAG "ENV1" "ENV2" ... -- kernel-trace timings of scripts/kbench.py
# under each environment setting (space-separated VAR=VALUE lists); stops at
# the first failure.  Run via gpurun from the repo root.
set -e -o pipefail
TAG=$1; shift
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  n=$(echo "$v" | tr ' =' '__')
  env $v timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d "$R/gpurun_out/${TAG}_$n" -o run -- \
      python3 "$R/scripts/kbench.py" --iters 10 > "$R/gpurun_out/${TAG}_$n.log" 2>&1
done
echo "variants $TAG done"
