#!/bin/bash
# Counter passes over one SpMM launch at a narrow (76-float, the P = 8
# feature block) and a 128-float width over all Reddit-shape rows
# (scripts/narrow_pass.py --only W): instructions per kind, SQ cycle shares,
# TA/TD busy and stalls, bytes beyond L2 and the L2 hit rate.  One rocprofv3
# run per counter set, each under its own time limit, chained so a failure
# stops the session; per-kernel means per dispatch by scripts/sq_counters.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$(pwd)
O=$R/gpurun_out/narrow_diag
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
pass() {
  local w=$1 name=$2; shift 2
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$O/w${w}_$name" -o p \
    -- python3 "$R/scripts/narrow_pass.py" --only "$w" --loops 20 > "$O/w${w}_$name.log" 2>&1
  local rc=$?
  echo "[w$w $name] rc=$rc"
  [ $rc -eq 0 ] && python3 "$R/scripts/sq_counters.py" "$O/w${w}_$name" > "$O/w${w}_$name.summary" 2>&1
  return $rc
}
for W in ${WIDTHS:-76 128}; do
  pass $W sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
      SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAVES &&
    pass $W insts SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE &&
    pass $W ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_LOAD_WAVEFRONT_sum GRBM_GUI_ACTIVE &&
    pass $W fetch FETCH_SIZE &&
    pass $W l2 TCC_HIT_sum TCC_MISS_sum || exit $?
done
