#!/bin/bash
# gpu_sq.sh TAG [LIB] [SET] -- counters of the serving step's stream coder
# (k_gc_roundtrip over 2 x 1408 C3 streams, no host frames, one step), one
# rocprofv3 --pmc pass per call, within one pass's limits:
#   SET issue (default): 8 SQ instruction / wait counters + 2 GRBM
#   SET fetch:           instruction fetch and issue-wait counters (8 SQ) + GRBM
#   SET icache:          the SQC instruction cache (4) + GRBM
#   SET fetch_size / write_size: HBM bytes, one TCC counter per pass (the level
#                        kernels' traffic per dispatch: profiles/pmc_fwd_l0_batch.json)
# LIB: another build of the library (RIC_AMD_LIB; "-" the tree's).  Time-limited.
set -e -o pipefail
TAG=$1
R=$(pwd)
OUT=$R/gpurun_out
mkdir -p "$OUT"
if [ -n "$2" ] && [ "$2" != "-" ]; then export RIC_AMD_LIB="$R/$2"; fi
case "${3:-issue}" in
  issue)  C="SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT" ;;
  fetch)  C="SQ_WAIT_INST_ANY SQ_IFETCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE" ;;
  icache) C="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ GRBM_GUI_ACTIVE" ;;
  fetch_size) C="FETCH_SIZE" ;;       # HBM reads (TCC: 3 counters), its own pass
  write_size) C="WRITE_SIZE" ;;       # HBM writes (TCC: 2 counters), its own pass
  *) echo "unknown counter set $3"; exit 2 ;;
esac
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc $C -f csv -d "$OUT/${TAG}_sq" -o run -- \
    python3 "$R/bench.py" --steps 1 --warmup 0 --n-host 0 --no-verify --no-cpu-baseline --no-latency \
    > "$OUT/${TAG}_sq.log" 2>&1
echo "sq $TAG done"
