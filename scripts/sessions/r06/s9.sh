#!/bin/bash
# round 6 session 9: the public call's rehearsal with the IPC exchange, P = 4, 8, twice
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
O=gpurun_out/r06_s9
mkdir -p $O
for r in 1 2; do
  timeout -k 10 600 python -u scripts/replicated_rehearsal.py --exchange ipc --P 4,8 --reps 5 > $O/rehearsal_ipc_$r.log 2>&1 || exit 1
done
grep -h summary $O/rehearsal_ipc_*.log | python -c "
import json, sys
for l in sys.stdin:
    d = json.loads(l); print(d['P'], {k: round(v, 2) for k, v in d['projected_speedup'].items()}, d['replication_local_ms_max'])"
