#!/bin/bash
# r5_run.sh TAG [steps] -- on the GPU box (via gpurun): the host coder A/B
# (scripts/hostbench binaries, pinned cores), a short C3 bench, and the
# two-rank gloo rehearsal of the stream gather on one GPU.  Skip parts with
# SKIP_AB / SKIP_BENCH / SKIP_W2.
set -e -o pipefail
TAG=$1
STEPS=${2:-3}
OUT=gpurun_out
mkdir -p "$OUT"
if [ -z "$SKIP_AB" ] && [ -n "$AB_BINS" ]; then
  timeout -k 10 300 bash scripts/hostbench/ab.sh $AB_BINS > "$OUT/${TAG}_ab.log" 2>&1
fi
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 700 python3 -u bench.py --steps "$STEPS" --warmup 2 $BENCH_ARGS > "$OUT/${TAG}_bench.log" 2> "$OUT/${TAG}_bench.err"
fi
if [ -z "$SKIP_W2" ]; then
  RIC_BENCH_BACKEND=gloo OMP_NUM_THREADS=8 timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 \
    --pool 448 --slots 8 --no-cpu-baseline --no-latency > "$OUT/${TAG}_w2.log" 2> "$OUT/${TAG}_w2.err"
fi
echo "run $TAG done"
