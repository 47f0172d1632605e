#!/bin/bash
# round 6 session 20 (TAG b: the shards' torch ops warmed by the loaders): where the first multi-rank call's extra time goes -- P
# ranks sharing the GPU at full Reddit shape, set-up stages traced
# (SGC_AMD_SETUP_TRACE=1: each stage synchronises the device around itself)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
O=gpurun_out/r06_s20${TAG:-}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 SGC_AMD_SETUP_TRACE=1
for P in 2 4 8; do
  mkdir -p $O/p$P
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$P \
     --master-addr=127.0.0.1 --master-port=$((29800+P)) tests/rank_precompute.py $O/p$P 232965 \
     > $O/p$P.log 2>&1 || { tail $O/p$P.log; exit 1; }
  python3 -c "
import json
for r in range($P):
    d = json.load(open('$O/p$P/rank%d.json' % r))
    print($P, r, [round(s, 4) for s in d['call_seconds']], d.get('ingest_seconds'), d.get('setup_seconds'))"
done
