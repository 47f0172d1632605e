#!/bin/bash
# Diagnostic counter passes on the Reddit-shape propagate() workload
# (scripts/pmc_traffic.py workload): SQ issue/wait shares, TA/TD busy and
# stalls, L1 TLB (UTCL1) hits and misses, TCP stalls.  One rocprofv3 run per
# counter set (MI355X_MICROARCH.md: per-block slot limits), each under its own
# time limit, chained so a failure stops the session; summaries by
# scripts/sq_counters.py (per-kernel mean per dispatch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$(pwd)
O=$R/gpurun_out/diag
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$O/$name" -o p \
    -- python3 "$R/scripts/pmc_traffic.py" workload "${DIAG_SHAPE:-reddit}" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  [ $rc -eq 0 ] && python3 "$R/scripts/sq_counters.py" "$O/$name" > "$O/$name.summary" 2>&1
  return $rc
}
pass tlb TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum &&
  pass ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_LOAD_WAVEFRONT_sum GRBM_GUI_ACTIVE &&
  pass tcp TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum
