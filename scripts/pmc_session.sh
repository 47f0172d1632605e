#!/bin/bash
# PMC traffic passes for the Reddit-shape hop (scripts/pmc_traffic.py), one
# counter set per rocprofv3 run, kernel trace only beside the counters; each
# pass under its own time limit, chained so a failure stops the session.
# Summarise afterwards on the host:
#   python scripts/pmc_traffic.py summarize gpurun_out/<tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$(pwd)
O=$R/gpurun_out/${PMC_TAG:-pmc}
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d "$O/$name" -o p \
    -- python3 "$R/scripts/pmc_traffic.py" workload > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  return $rc
}
pass pmc_fetch FETCH_SIZE &&
  pass pmc_write WRITE_SIZE &&
  pass pmc_l2 TCC_HIT_sum TCC_MISS_sum
