#!/bin/bash
# round 6 session 21: classifier forward with each finished tile stored at once
# by stores the compiler's wait counting does not see (variants/lin_asm,
# SGC_SPLIT_ASM_STORES=1) against the held tiles (default): parity tests on
# the variant first, then interleaved timing and kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
R=$(pwd)
O=$R/gpurun_out/r06_s21${TAG:-}
mkdir -p $O
export PYTHONPATH=$R
SGC_AMD_LIB=$R/variants/lin_asm/libsgc_amd.so timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "linear or SGC or logits or nonfinite" > $O/tests_asm.log 2>&1
rc=$?; tail -2 $O/tests_asm.log; [ $rc = 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in default lin_asm; do
    lib=$R/sgc_amd/libsgc_amd.so; [ $v != default ] && lib=$R/variants/$v/libsgc_amd.so
    SGC_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_$rep -o p \
      -- python3 $R/scripts/linear_ab.py --kernels 5 --rounds 3 > $O/${v}_$rep.log 2>&1 || exit 1
    python3 - <<PY
import csv, glob
f = glob.glob("$O/${v}_$rep/**/*kernel_stats.csv", recursive=True)[0]
print("$v rep$rep", [l.strip()[:150] for l in open("$O/${v}_$rep.log") if "ms" in l or "err" in l][-2:],
      [(r["Name"].split("(")[0][-30:], round(float(r["AverageNs"]) / 1000, 2))
       for r in csv.DictReader(open(f)) if "linear_split" in r["Name"]])
PY
  done
done
