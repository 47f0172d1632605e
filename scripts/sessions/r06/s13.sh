#!/bin/bash
# round 6 session 13: column-block backward -- row ranges 48 (default) / 40 /
# 64 interleaved under kernel stats, then SQ and traffic counters of the default
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
R=$(pwd)
O=$R/gpurun_out/r06_s13${TAG:-}
mkdir -p $O
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for v in default cols_r40 cols_r64; do
    lib=$R/sgc_amd/libsgc_amd.so; [ $v != default ] && lib=$R/variants/$v/libsgc_amd.so
    SGC_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_$rep -o p \
      -- python3 $R/scripts/bwd_ab.py --kernel 0 > $O/${v}_$rep.log 2>&1 || exit 1
    python3 - <<PY
import csv, glob, json
f = glob.glob("$O/${v}_$rep/**/*kernel_stats.csv", recursive=True)[0]
rec = [json.loads(l) for l in open("$O/${v}_$rep.log") if l.startswith("{")][0]
print("$v rep$rep", round(rec["backward_ms"], 4), rec["rel_err"],
      [(r["Name"].split("(")[0][-40:], round(float(r["AverageNs"]) / 1000, 2))
       for r in csv.DictReader(open(f)) if "xent" in r["Name"]])
PY
  done
done
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$O/$name" -o p \
    -- python3 "$R/scripts/bwd_ab.py" --kernel 0 > "$O/$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] && (cd "$R" && python3 scripts/sq_counters.py "$O/$name") > "$O/$name.summary" 2>&1
  return $rc
}
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_VMEM SQ_WAVES SQ_BUSY_CYCLES &&
pass insts SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES \
    SQ_INSTS_LDS SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE &&
pass fetch FETCH_SIZE &&
pass l2 TCC_HIT_sum TCC_MISS_sum || exit 1
grep -h "xent_dw_cols" $O/*.summary
