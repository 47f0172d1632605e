#!/bin/bash
# round 6 session 10: the first sgc_precompute's timeline (kernel + HIP API trace)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
R=$(pwd)
O=$R/gpurun_out/r06_s10${TAG:-}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/trace -o p \
  -- python3 $R/scripts/first_call_stages.py > $O/stages.log 2>&1
rc=$?; grep "{" $O/stages.log; exit $rc
cd $R && timeout -k 10 300 python -u scripts/first_call.py --warm > $O/first_call.log 2>&1 && grep "{" $O/first_call.log
