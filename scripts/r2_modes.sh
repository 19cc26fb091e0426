#!/bin/bash
# r2_modes.sh TAG -- the C4 and C5 bench workloads on one GPU, then a 2-rank
# gloo rehearsal of C4 and C3 (both ranks on this GPU).  Each step has its
# own limit; stop at the first failure.
TAG=${1:-r2m}
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
export MASTER_ADDR=127.0.0.1
run() { local name=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/${TAG}_${name}.log" 2>&1; local rc=$?
  echo "$name rc=$rc"; tail -1 "$OUT/${TAG}_${name}.log" | cut -c1-1500
  [ $rc -eq 0 ] || exit $rc; }
run c4 300 python3 -u bench.py --workload C4 --steps 2 --warmup 1 --no-cpu-baseline
run c5 300 python3 -u bench.py --workload C5 --steps 2 --warmup 1 --no-cpu-baseline
run c4w2 300 env RIC_BENCH_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload C4 --steps 2 --warmup 1 --threads 8
run c3w2 300 env RIC_BENCH_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 1 --warmup 1 --threads 8 --frames 16
echo "modes $TAG done"
