#!/bin/bash
# Round-5 session 8: classifier backward with 512 (default) / 256 / 1024 dW partial slabs, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
rm -f gpurun_out/bwd_ab.log
for r in 1 2 3; do
  for L in sgc_amd/libsgc_amd.so variants/lib_s256.so variants/lib_s1024.so; do
    SGC_AMD_LIB=$L timeout -k 10 120 python scripts/bwd_ab.py >> gpurun_out/bwd_ab.log 2>&1 || exit $?
  done
done
