#!/bin/bash
# Round-5 session 11: split classifier W fill kk-major (conflict-free LDS writes, default)
# vs granule order (variants/lib_prevfill.so): linear tests, then interleaved timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py -x -q -k "linear" --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/lin_tests_s11.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/lin_tests_s11.log
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/linear_ab_s11.log
for r in 1 2 3; do
  for L in sgc_amd/libsgc_amd.so variants/lib_prevfill.so; do
    echo "== $L" >> gpurun_out/linear_ab_s11.log
    SGC_AMD_LIB=$L timeout -k 10 120 python scripts/linear_ab.py --kernels 5 --rounds 3 >> gpurun_out/linear_ab_s11.log 2>&1 || exit $?
  done
done
