#!/bin/bash
# s4_w2.sh TAG -- the default bench (balanced split) on one GPU, then a 2-rank
# gloo rehearsal of it on the same GPU (small coder launches); each step under
# its own limit, stop at the first failure.
TAG=${1:-s4w2}
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
export MASTER_ADDR=127.0.0.1
run() { local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/${TAG}_${name}.log" 2> "$OUT/${TAG}_${name}.err"; local rc=$?
  echo "$name rc=$rc"; tail -1 "$OUT/${TAG}_${name}.log" | cut -c1-300
  [ $rc -eq 0 ] || exit $rc; }
run n1 300 python3 -u bench.py --steps 2 --warmup 2 --no-cpu-baseline
run w2 300 env RIC_BENCH_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 1 --warmup 2 --threads 8 --pool 16
echo "w2 $TAG done"
