#!/bin/bash
# round 6 session 14: column-block backward with interleaved classes (one
# 12-B dY load per row) and 16-deep reduction batches: parity tests, then
# kernel stats (3 runs) and SQ counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
R=$(pwd)
O=$R/gpurun_out/r06_s14${TAG:-}
mkdir -p $O
export PYTHONPATH=$R
timeout -k 10 120 python3 $R/scripts/bwd_ab.py --kernel 0 > $O/first.log 2>&1 || { cat $O/first.log; exit 1; }
cat $O/first.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "linear_backward or closure or lbfgs or cross_entropy or xent" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for rep in 1 2 3; do
  for k in 0 1; do
    timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/k${k}_$rep -o p \
      -- python3 $R/scripts/bwd_ab.py --kernel $k > $O/k${k}_$rep.log 2>&1 || exit 1
    python3 - <<PY
import csv, glob, json
f = glob.glob("$O/k${k}_$rep/**/*kernel_stats.csv", recursive=True)[0]
rec = [json.loads(l) for l in open("$O/k${k}_$rep.log") if l.startswith("{")][0]
print("k$k rep$rep", round(rec["backward_ms"], 4), rec["rel_err"],
      [(r["Name"].split("(")[0][-40:], round(float(r["AverageNs"]) / 1000, 2))
       for r in csv.DictReader(open(f)) if "xent" in r["Name"]])
PY
  done
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_VMEM SQ_WAVES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $O/sq -o p \
    -- python3 $R/scripts/bwd_ab.py --kernel 0 > $O/sq.log 2>&1 &&
  (cd $R && python3 scripts/sq_counters.py $O/sq) > $O/sq.summary 2>&1
grep -h "xent_dw_cols" $O/sq.summary
