#!/bin/bash
# round 6 session 7: kernel times of the two weight-backward kernels (stats)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
R=$(pwd)
O=$R/gpurun_out/r06_s7${TAG:-}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
for k in 1 2; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_k$k -o p \
    -- python3 $R/scripts/bwd_ab.py --kernel $k > $O/stats_k$k.log 2>&1 || exit 1
  grep "{" $O/stats_k$k.log
  python3 - <<PY
import csv, glob
f = glob.glob("$O/stats_k$k/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print($k, r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1000, 2), "us")
PY
done
cd $R && timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "linear_backward or closure or lbfgs or logits or cross_entropy or nonfinite" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
