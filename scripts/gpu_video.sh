#!/bin/bash
# gpu_video.sh TAG [ENV=VAL ...] -- the video path on the GPU in one gpurun
# call: the video parity tests, scripts/video_bench.py (frames/s), its kernel
# trace (per-kernel time and HBM fraction) and the FETCH_SIZE / WRITE_SIZE
# passes (separate runs), summarised into gpurun_out/TAG_kernels.json.
# Extra ENV=VAL arguments are exported first (A/B knobs such as RIC_OBMC_RW).
set -e -o pipefail
TAG=$1; shift
for kv in "$@"; do export "$kv"; done
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
ARGS="--w 1920 --h 1080 --frames 30 --q 20"
if [ -z "$NO_TESTS" ]; then
    timeout -k 10 400 python3 -u -m pytest tests/test_gpu_video.py -m gpu -x -v --timeout 120 --timeout-method thread \
        > "$OUT/${TAG}_tests.log" 2>&1
fi
timeout -k 10 300 python3 -u scripts/video_bench.py $ARGS --cpu-frames 0 > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/${TAG}_kt" -o run -- \
    python3 "$R/scripts/video_bench.py" $ARGS --cpu-frames 0 > "$OUT/${TAG}_kt.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d "$OUT/${TAG}_pf" -o run -- \
    python3 "$R/scripts/video_bench.py" $ARGS --cpu-frames 0 > "$OUT/${TAG}_pf.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d "$OUT/${TAG}_pw" -o run -- \
    python3 "$R/scripts/video_bench.py" $ARGS --cpu-frames 0 > "$OUT/${TAG}_pw.log" 2>&1
cd "$R"
KS=$(find "$OUT/${TAG}_kt" -name 'run_kernel_stats.csv' | head -1)
PF=$(find "$OUT/${TAG}_pf" -name 'run_counter_collection.csv' | head -1)
PW=$(find "$OUT/${TAG}_pw" -name 'run_counter_collection.csv' | head -1)
python3 scripts/video_bench.py $ARGS --kstats "$KS" --pmc "$PF" "$PW" > "$OUT/${TAG}_kernels.json"
echo "video $TAG done"
