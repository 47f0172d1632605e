#!/bin/bash
# round 6 session 8: split-bf16 weight backward slab geometry (steps x phases)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
R=$(pwd)
O=$R/gpurun_out/r06_s8${TAG:-}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
for v in default split_s5_p2 split_s8_p1 split_s6_p1; do
  lib=$R/sgc_amd/libsgc_amd.so; [ $v != default ] && lib=$R/variants/$v/libsgc_amd.so
  for k in 1 2; do
    [ $v != default ] && [ $k = 1 ] && continue
    SGC_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_k$k -o p \
      -- python3 $R/scripts/bwd_ab.py --kernel $k > $O/${v}_k$k.log 2>&1 || exit 1
    python3 - <<PY
import csv, glob, json
f = glob.glob("$O/${v}_k$k/**/*kernel_stats.csv", recursive=True)[0]
rec = [l for l in open("$O/${v}_k$k.log") if l.startswith("{")]
print("$v k$k", json.loads(rec[0])["backward_ms"] if rec else None,
      [(r["Name"].split("(")[0][-40:], round(float(r["AverageNs"]) / 1000, 2))
       for r in csv.DictReader(open(f)) if "xent" in r["Name"]])
PY
  done
done
cd $R && timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "linear_backward or closure or lbfgs or logits or cross_entropy or nonfinite" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
