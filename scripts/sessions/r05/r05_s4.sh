#!/bin/bash
# Round-5 session 4: classifier store variants (held 6 vs 1), 3 interleaved rounds each
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
rm -f gpurun_out/linear_ab_s4.log
for L in sgc_amd/libsgc_amd.so variants/lib_h1.so sgc_amd/libsgc_amd.so variants/lib_h1.so; do
  echo "== $L" >> gpurun_out/linear_ab_s4.log
  SGC_AMD_LIB=$L timeout -k 10 120 python scripts/linear_ab.py --kernels 5,6,7 --rounds 3 >> gpurun_out/linear_ab_s4.log 2>&1 || exit $?
done
SGC_AMD_LIB=sgc_amd/libsgc_amd.so timeout -k 10 150 python -u -m pytest tests/test_gpu_parity.py -x -q -k "linear" --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/lin_tests.log 2>&1
echo "tests rc=$?"
