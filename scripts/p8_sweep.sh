#!/bin/bash
# All multi-GPU pipeline variants of scripts/p8_rehearsal.py, one log each
# under gpurun_out/p8/ (every run under its own time limit).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
O=gpurun_out/p8; mkdir -p $O
run() { timeout -k 10 300 python scripts/p8_rehearsal.py --layouts ${LAYOUTS:-8x1,4x2,4x1,2x1} "$@" \
          > "$O/$(echo "$@" | tr ' -' '__').log" 2>&1; }
run --group-floats 0 && run --group-floats 0 --row-chunks 4 && run --group-floats 0 --row-chunks 8 &&
  run --group-floats 128 && run --group-floats 256
