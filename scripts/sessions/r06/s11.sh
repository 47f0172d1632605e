#!/bin/bash
# round 6 session 11: weight backward on split-bf16 column blocks
# (xent_dw_cols_kernel) -- parity tests, then the three kernels interleaved
# under rocprofv3 kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
R=$(pwd)
O=$R/gpurun_out/r06_s11${TAG:-}
mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 120 python3 $R/scripts/bwd_ab.py --kernel 0 > $O/first.log 2>&1 || { cat $O/first.log; exit 1; }
cat $O/first.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "linear_backward or closure or lbfgs or cross_entropy or xent" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for k in 0 1 2; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k${k}_$rep -o p \
      -- python3 $R/scripts/bwd_ab.py --kernel $k > $O/k${k}_$rep.log 2>&1 || exit 1
    python3 - <<PY
import csv, glob, json
f = glob.glob("$O/k${k}_$rep/**/*kernel_stats.csv", recursive=True)[0]
rec = [l for l in open("$O/k${k}_$rep.log") if l.startswith("{")]
print("k$k rep$rep", json.loads(rec[0])["backward_ms"] if rec else None, json.loads(rec[0])["rel_err"] if rec else None,
      [(r["Name"].split("(")[0][-40:], round(float(r["AverageNs"]) / 1000, 2))
       for r in csv.DictReader(open(f)) if "xent" in r["Name"]])
PY
  done
done
