#!/bin/bash
# Round-5 session 7: split classifier, held tiles stored as flat runs through LDS (default)
# vs in the MFMA layout (variants/lib_noflat.so), interleaved; then the linear tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
rm -f gpurun_out/linear_ab_s7.log
SGC_AMD_LIB=sgc_amd/libsgc_amd.so timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py -x -q -k "linear" --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/lin_tests_s7.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/lin_tests_s7.log
[ $rc -eq 0 ] || exit $rc
for L in sgc_amd/libsgc_amd.so variants/lib_noflat.so sgc_amd/libsgc_amd.so variants/lib_noflat.so sgc_amd/libsgc_amd.so variants/lib_noflat.so; do
  echo "== $L" >> gpurun_out/linear_ab_s7.log
  SGC_AMD_LIB=$L timeout -k 10 120 python scripts/linear_ab.py --kernels 5 --rounds 3 >> gpurun_out/linear_ab_s7.log 2>&1 || exit $?
done
