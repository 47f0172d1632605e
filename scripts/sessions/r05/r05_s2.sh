#!/bin/bash
# Round-5 session 2: classifier idle-wave experiment, replicated rehearsal
# (two-stream 1:3:3:1 chunks), multi-GPU tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
( while sleep 45; do date +%T >> gpurun_out/heartbeat.log; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for L in sgc_amd/libsgc_amd.so variants/lib_idle.so; do
  SGC_AMD_LIB=$L timeout -k 10 120 python scripts/linear_ab.py --kernels 5,7,8 --rounds 3 > gpurun_out/linear_ab_$(basename $L .so).log 2>&1 || exit $?
done
timeout -k 10 600 python scripts/replicated_rehearsal.py > gpurun_out/replicated_rehearsal.log 2>&1 || exit $?
timeout -k 10 700 python -u -m pytest tests/test_gpu_multigpu.py -x -v -m "gpu and not slow" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/mgpu_tests.log 2>&1
echo "mgpu rc=$?"
echo done
