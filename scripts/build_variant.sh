#!/bin/bash
# build_variant.sh OUT.so SRC.hip FLAGS... -- a variant of the library for A/B
# runs (scripts/gpu_ab.sh): SRC recompiled with FLAGS (e.g. -DRIC_GC_ELOW_V=1),
# linked with the tree's other objects (build the tree first).  CPU only.
set -e
OUT=$1; SRC=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/rududu-image-codec_amd
B=$(basename "$SRC")
T=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fwrapv -I"$R/include" -I"$P/csrc" "$@" -c "$P/csrc/$B" -o "$T/$B.o"
objs=$(ls "$P"/build/*.o | grep -v "/$B.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs "$T/$B.o" -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o "$OUT"
rm -rf "$T"
echo "built $OUT"
