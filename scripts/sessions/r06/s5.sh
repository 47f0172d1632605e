#!/bin/bash
# round 6 session 5: counters of the two weight-backward kernels (bwd_ab.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
R=$(pwd)
O=$R/gpurun_out/r06_s5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
pass() {
  local name=$1 k=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$O/$name" -o p \
    -- python3 "$R/scripts/bwd_ab.py" --kernel $k > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  [ $rc -eq 0 ] && (cd "$R" && python3 scripts/sq_counters.py "$O/$name") > "$O/$name.summary" 2>&1
  return $rc
}
for k in 1 2; do
  pass sq_k$k $k SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
      SQ_ACTIVE_INST_VMEM SQ_WAVES SQ_BUSY_CYCLES || exit 1
  pass insts_k$k $k SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES \
      SQ_INSTS_SALU SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE || exit 1
  pass tcp_k$k $k TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE || exit 1
done
grep -h "xent_dw" $O/*.summary
