#!/bin/bash
# PMC traffic passes for one shape's propagate() (scripts/pmc_traffic.py), one
# counter set per rocprofv3 run, kernel trace only beside the counters; each
# pass under its own time limit, chained so a failure stops the session, then
# the summary (-> profiles/pmc_<shape>.json, merged back with gpurun_out).
#   PMC_SHAPE=reddit|rmat  PMC_TAG=<dir name under gpurun_out>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$(pwd)
SHAPE=${PMC_SHAPE:-reddit}
O=$R/gpurun_out/${PMC_TAG:-pmc_$SHAPE}
mkdir -p "$O"
export PMC_META=$O/meta.json
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$O/$name" -o p \
    -- python3 "$R/scripts/pmc_traffic.py" workload "$SHAPE" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$SHAPE $name] rc=$rc"
  return $rc
}
pass pmc_fetch FETCH_SIZE &&
  pass pmc_write WRITE_SIZE &&
  pass pmc_l2 TCC_HIT_sum TCC_MISS_sum &&
  python3 "$R/scripts/pmc_traffic.py" summarize "$O" "$SHAPE" > "$O/summary.log" 2>&1 &&
  cp "$R/profiles/pmc_$SHAPE.json" "$O/pmc_$SHAPE.json"
