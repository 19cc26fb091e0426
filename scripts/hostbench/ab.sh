#!/bin/bash
# ab.sh BIN... -- CPU A/B timing of host-coder builds on the GPU box's host
# (each binary pinned to one core, interleaved rounds).
set -e -o pipefail
R=$(pwd)
python3 "$R/scripts/hostbench/dump_c3.py" /tmp/c3_bands.bin
for round in 1 2 3; do
  for b in "$@"; do
    echo "== $b round $round"
    timeout -k 5 120 taskset -c 2 "$R/scripts/hostbench/$b" /tmp/c3_bands.bin 3
  done
done
