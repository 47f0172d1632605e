#!/bin/bash
# Round-5 session 10: split classifier ring depth 4 (templated slots) / previous hand-unrolled 4 / 6 / 8,
# interleaved (kernels 5 = full, 7 = loads + exchange only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
rm -f gpurun_out/linear_ab_s10.log
for r in 1 2; do
  for L in sgc_amd/libsgc_amd.so variants/lib_old.so variants/lib_d6.so variants/lib_d8.so; do
    echo "== $L" >> gpurun_out/linear_ab_s10.log
    SGC_AMD_LIB=$L timeout -k 10 120 python scripts/linear_ab.py --kernels 5,7 --rounds 3 >> gpurun_out/linear_ab_s10.log 2>&1 || exit $?
  done
done
