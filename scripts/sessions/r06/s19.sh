#!/bin/bash
# round 6 session 19: the fused training step (sgc_linear_xent_f32) on the
# column-block dW -- parity tests, then the classifier record
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
R=$(pwd)
O=$R/gpurun_out/r06_s19${TAG:-}
mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_e2e.py -k "xent or cross_entropy or closure or lbfgs or linear_backward" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python -m sgc_amd.classifier_bench > $O/classifier.log 2>&1 || { tail $O/classifier.log; exit 1; }
python3 -c "
import json; d=json.loads([l for l in open('$O/classifier.log') if l.startswith('{')][-1])
print('fwd', d['forward']['ms'], 'bwd', d['backward']['ms'], d['closure'], d['lbfgs'])"
