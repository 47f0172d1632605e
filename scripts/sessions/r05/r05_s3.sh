#!/bin/bash
# Round-5 session 3: storer-wave classifier variant (tests first, time-limited),
# replicated rehearsal with hub-aware chunk order.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
( while sleep 45; do date +%T >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
SGC_AMD_LIB=variants/lib_storer.so timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py -x -q -k "linear" --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/lin_tests_storer.log 2>&1
rc=$?; echo "storer tests rc=$rc"; [ $rc -gt 1 ] && exit $rc
for L in sgc_amd/libsgc_amd.so variants/lib_storer.so sgc_amd/libsgc_amd.so variants/lib_storer.so; do
  SGC_AMD_LIB=$L timeout -k 10 120 python scripts/linear_ab.py --kernels 5,6,7 --rounds 3 >> gpurun_out/linear_ab_storer.log 2>&1 || exit $?
done
timeout -k 10 600 python scripts/replicated_rehearsal.py > gpurun_out/replicated_rehearsal.log 2>&1 || exit $?
echo done
