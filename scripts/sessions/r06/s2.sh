#!/bin/bash
# round 6 session 2: first-call anatomy (allocation reserve), the replicated
# rehearsal with the IPC exchange vs the collective one
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
O=gpurun_out/r06_s2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 0 4 8; do
  timeout -k 10 240 python -u scripts/first_call.py --warm --reserve-gb $r >> $O/first_call.log 2>&1 || exit 1
done
timeout -k 10 900 python -u scripts/replicated_rehearsal.py --exchange ipc --P 2,4,8 --reps 5 > $O/rehearsal_ipc.log 2>&1 &&
timeout -k 10 900 python -u scripts/replicated_rehearsal.py --exchange collective --P 8 --reps 5 > $O/rehearsal_coll.log 2>&1
rc=$?
echo "rc=$rc"
grep summary $O/rehearsal_*.log
exit $rc
