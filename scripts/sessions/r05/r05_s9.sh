#!/bin/bash
# Round-5 session 9: split-bf16 classifier backward (linear_bwd 2) vs the fp32 slab kernel (1):
# linear tests, then interleaved timing, then a kernel trace for registers / scratch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "linear_backward or sgc_model or closure or fused_loss or lbfgs" --timeout 60 --timeout-method thread -p no:cacheprovider > gpurun_out/bwd_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/bwd_tests.log
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/bwd_ab2.log
for r in 1 2 3; do
  for b in 1 2; do
    timeout -k 10 120 python scripts/bwd_ab.py --bwd $b >> gpurun_out/bwd_ab2.log 2>&1 || exit $?
  done
done
grep '^{' gpurun_out/bwd_ab2.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/bwdtrace -o p -- python3 $GRAFT_REPO_ROOT/scripts/bwd_ab.py --bwd 2 > /dev/null 2>&1
echo "trace rc=$?"
