#!/bin/bash
# r6_ab.sh TAG "ENV_A" "ENV_B" ... -- the whole GPU suite (SKIP_ALL=1: not),
# then one short C3 bench per environment setting ("-" = none).  Via gpurun.
set -e -o pipefail
TAG=$1; shift
OUT=gpurun_out
mkdir -p "$OUT"
if [ -z "$SKIP_ALL" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/${TAG}_all.log" 2>&1
  echo "suite: $(tail -1 $OUT/${TAG}_all.log)"
fi
i=0
for e in "$@"; do
  i=$((i+1))
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 400 python3 -u bench.py --steps ${STEPS:-2} --warmup 2 --no-cpu-baseline --no-latency --no-split \
      > "$OUT/${TAG}_b$i.log" 2> "$OUT/${TAG}_b$i.err"
  python3 - "$OUT/${TAG}_b$i.log" "$e" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(l)
sc = d.get("stream_coder", {})
print("[%s] value %.1f ms_per_step %.1f frames %s roofline %.4f launch %s verified %s" % (
    sys.argv[2], d["value"], d["ms_per_step"], d["config"].get("frames_per_gpu_per_step"), d["roofline"]["frac"],
    sc.get("encode_then_decode", {}).get("ms_per_launch"), d.get("verified")))
PY
done
