#!/bin/bash
# round 6 session 3: first-call stages (one GPU), the public call's first vs
# steady calls with P ranks sharing the GPU at full Reddit shape
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
O=gpurun_out/r06_s3
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/first_call_stages.py > $O/stages.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/first_call_stages.py --reserve-gb 8 >> $O/stages.log 2>&1 || exit 1
for P in 2 4 8; do
  mkdir -p $O/p$P
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$P \
     --master-addr=127.0.0.1 --master-port=$((29700+P)) tests/rank_precompute.py $O/p$P 232965 \
     > $O/p$P.log 2>&1 || exit 1
  cat $O/p$P/rank0.json; echo
done
# the classifier kernels' counters, labelled (scripts/sq_counters.py fixed)
bash scripts/pmc_classifier.sh > $O/pmc_cls.log 2>&1
rc=$?
mkdir -p $O/pmc_cls && cp gpurun_out/pmc_cls/*.summary $O/pmc_cls/ 2>/dev/null
exit $rc
