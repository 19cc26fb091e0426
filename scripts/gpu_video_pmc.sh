#!/bin/bash
# gpu_video_pmc.sh TAG "COUNTERS1" ["COUNTERS2" ...] -- one rocprofv3 --pmc pass
# per argument over scripts/video_bench.py (1080p, 30 frames); summarise the
# per-dispatch counters of the video kernels with scripts/pmc_table.py.
set -e -o pipefail
TAG=$1; shift
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
k=0
for ctrs in "$@"; do
  k=$((k+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -f csv -d "$R/gpurun_out/${TAG}_p$k" -o run -- \
      python3 "$R/scripts/video_bench.py" --cpu-frames 0 > "$R/gpurun_out/${TAG}_p$k.log" 2>&1
done
echo "video pmc $TAG done"
