#!/bin/bash
# Counter passes over the classifier kernels (sgc_amd.classifier_bench
# --workload: sgc_linear_f32 and sgc_linear_backward_f32 at Reddit-train
# shape), one rocprofv3 run per counter set, each time-limited; per-kernel
# means by scripts/sq_counters.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$(pwd)
O=$R/gpurun_out/pmc_cls
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$O/$name" -o p \
    -- python3 -m sgc_amd.classifier_bench --workload > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  [ $rc -eq 0 ] && (cd "$R" && python3 scripts/sq_counters.py "$O/$name") > "$O/$name.summary" 2>&1
  return $rc
}
export PYTHONPATH=$R
pass sq SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
    SQ_ACTIVE_INST_LDS SQ_WAVES SQ_BUSY_CYCLES &&
  pass insts SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES \
    SQ_INSTS_SALU GRBM_GUI_ACTIVE &&
  pass lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE &&
  pass fetch FETCH_SIZE || exit $?
