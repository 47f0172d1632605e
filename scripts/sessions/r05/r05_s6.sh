#!/bin/bash
# Round-5 session 6: split-bf16 classifier with 8 / 12 / 16 waves per CU, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
rm -f gpurun_out/linear_ab_s6.log
for L in sgc_amd/libsgc_amd.so variants/lib_w12.so variants/lib_w16.so sgc_amd/libsgc_amd.so variants/lib_w12.so variants/lib_w16.so; do
  echo "== $L" >> gpurun_out/linear_ab_s6.log
  SGC_AMD_LIB=$L timeout -k 10 120 python scripts/linear_ab.py --kernels 5,6,7 --rounds 3 >> gpurun_out/linear_ab_s6.log 2>&1 || exit $?
done
