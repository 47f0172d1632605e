#!/bin/bash
# round 6 session 6: kernel times (rocprofv3 --stats) and counters of the two
# weight-backward kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
R=$(pwd)
O=$R/gpurun_out/r06_s6${TAG:-}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
for k in 1 2; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_k$k -o p \
    -- python3 $R/scripts/bwd_ab.py --kernel $k > $O/stats_k$k.log 2>&1 || exit 1
done
pass() {
  local name=$1 k=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$O/$name" -o p \
    -- python3 "$R/scripts/bwd_ab.py" --kernel $k > "$O/$name.log" 2>&1
  local rc=$?
  [ $rc -eq 0 ] && (cd "$R" && python3 scripts/sq_counters.py "$O/$name") > "$O/$name.summary" 2>&1
  return $rc
}
pass sq_k2 2 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_VMEM SQ_WAVES SQ_BUSY_CYCLES &&
pass insts_k2 2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES \
    SQ_INSTS_LDS SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE || exit 1
for k in 1 2; do
  f=$(find $O/stats_k$k -name "*kernel_stats.csv" | head -1); echo "== k$k"; cut -d, -f1-5 $f | head -8
done
grep -h "xent_dw" $O/*.summary
