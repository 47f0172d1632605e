#!/bin/bash
# round 6 session 24: column-block backward with two column blocks per workgroup (8 waves, 512 contiguous bytes of each row; variants/h2) and the loads-only forms of both
# against the default; interleaved runs, kernel stats; parity of h2
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
R=$(pwd)
O=$R/gpurun_out/r06_s24${TAG:-}
mkdir -p $O
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in default h2 diag1 h2_diag1; do
    lib=$R/sgc_amd/libsgc_amd.so; [ $v != default ] && lib=$R/variants/$v/libsgc_amd.so
    SGC_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_$rep -o p \
      -- python3 $R/scripts/bwd_ab.py --kernel 0 > $O/${v}_$rep.log 2>&1 || exit 1
    python3 - <<PY
import csv, glob, json
f = glob.glob("$O/${v}_$rep/**/*kernel_stats.csv", recursive=True)[0]
print("$v rep$rep", [(r["Name"].split("(")[0][-40:], round(float(r["AverageNs"]) / 1000, 2))
       for r in csv.DictReader(open(f)) if "xent" in r["Name"]])
PY
  done
done
cd $R && SGC_AMD_LIB=$R/variants/h2/libsgc_amd.so timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "linear_backward" > $O/tests_h2.log 2>&1
rc=$?; tail -2 $O/tests_h2.log; exit $rc
