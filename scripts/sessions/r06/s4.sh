#!/bin/bash
# round 6 session 4: split-bf16 weight backward -- A/B against the fp32 slabs,
# two register budgets, and the classifier tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
O=gpurun_out/r06_s4${TAG:-}
mkdir -p $O
for rep in 1 2; do
  for k in 1 2; do
    timeout -k 10 120 python -u scripts/bwd_ab.py --kernel $k >> $O/bwd_ab.log 2>&1 || exit 1
  done
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "linear or backward or closure or lbfgs or logits or cross_entropy" > $O/tests.log 2>&1
rc=$?
grep "{" $O/bwd_ab.log
tail -3 $O/tests.log
exit $rc
