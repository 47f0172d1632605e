#!/bin/bash
# Round-5 session 1: classifier A/B + tests, pad A/B, replicated rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
( while sleep 45; do date +%T >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 120 python scripts/linear_ab.py --kernels 2,5,6,7,8 --rounds 3 > gpurun_out/linear_ab.log 2>&1 || exit $?
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "linear" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/lin_tests.log 2>&1
rc=$?; echo "lin_tests rc=$rc"; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python scripts/pad_ab.py > gpurun_out/pad_ab.log 2>&1 || exit $?
timeout -k 10 600 python scripts/replicated_rehearsal.py > gpurun_out/replicated_rehearsal.log 2>&1 || exit $?

timeout -k 10 200 python scripts/host_breakdown.py > gpurun_out/host_breakdown.log 2>&1

timeout -k 10 200 python scripts/combo_ab.py --shape pubmed --configs "base:;r4:rows_per_wave=4;r4x:rows_per_wave=4,xcd_slices=1;r2:rows_per_wave=2;r2x:rows_per_wave=2,xcd_slices=1" > gpurun_out/combo_pubmed.log 2>&1
echo done
