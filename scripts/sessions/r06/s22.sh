#!/bin/bash
# round 6 session 22: counters of the final library's classifier kernels
# (xent_dw_cols_kernel, its reduction, linear_split_kernel), one counter set
# per rocprofv3 run, kernel names in the summaries
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
R=$(pwd)
O=$R/gpurun_out/r06_s22${TAG:-}
mkdir -p $O
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$O/$name" -o p \
    -- python3 -m sgc_amd.classifier_bench --workload > "$O/$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] && (cd "$R" && python3 scripts/sq_counters.py "$O/$name") > "$O/$name.summary" 2>&1
  return $rc
}
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_VMEM SQ_WAVES SQ_BUSY_CYCLES &&
pass insts SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES \
    SQ_INSTS_LDS SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE &&
pass fetch FETCH_SIZE &&
pass write WRITE_SIZE || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o p \
    -- python3 -m sgc_amd.classifier_bench --workload > $O/stats.log 2>&1 || exit 1
grep -h "xent_dw_cols\|linear_split\|reduce_dw_db" $O/*.summary | cut -c1-400
