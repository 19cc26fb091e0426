#!/bin/bash
# gpu_ab.sh TAG STEPS VARIANT... -- the default bench once per variant, in
# order, for A/B comparisons within one box call.  VARIANT = LIB[@VAR=VAL,...]:
# LIB a library build (RIC_AMD_LIB; "-" = the tree's own), then environment
# settings for that run (e.g. -@RIC_GC_FUSE=0).  Every GPU step is
# time-limited; the first failure ends the script.
set -e -o pipefail
TAG=$1; STEPS=$2; shift 2
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
i=0
for V in "$@"; do
    L=${V%%@*}
    E=""
    if [ "$V" != "$L" ]; then E=${V#*@}; E=${E//,/ }; fi
    if [ "$L" = "-" ]; then LIB=""; else LIB="$R/$L"; fi
    env RIC_AMD_LIB="$LIB" $E timeout -k 10 400 python3 -u bench.py --steps "$STEPS" --no-cpu-baseline --no-latency \
        > "$OUT/${TAG}_$i.log" 2> "$OUT/${TAG}_$i.err"
    echo "variant $i: $V" >> "$OUT/${TAG}_variants.txt"
    i=$((i + 1))
done
echo "ab $TAG done"
