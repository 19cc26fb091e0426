#!/bin/bash
# lds_sweep.sh TAG [LDS...] -- the default C3 bench (GPU stream coder) with the
# coder waves' LDS footprint padded to each size (RIC_GC_LDS, 0 = none); each
# run under its own limit, stop at the first failure.
TAG=${1:-lds}; shift
SIZES=${@:-0 33792}
OUT=$(pwd)/gpurun_out
mkdir -p "$OUT"
for s in $SIZES; do
  RIC_GC_LDS=$s timeout -k 10 240 python3 -u bench.py --steps 2 --warmup 1 --no-cpu-baseline \
      > "$OUT/${TAG}_lds$s.log" 2> "$OUT/${TAG}_lds$s.err"
  rc=$?
  echo "lds $s rc=$rc"
  python3 - "$OUT/${TAG}_lds$s.log" <<'PY' || true
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d.get("verified"), json.dumps(d.get("stream_coder")))
PY
  [ $rc -eq 0 ] || exit $rc
done
echo "lds_sweep $TAG done"
