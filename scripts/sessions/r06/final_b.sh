#!/bin/bash
# round-6 final: PMC records of the final library, bench N=1 reading them,
# rocprofv3 stats of the bench; the public call's first vs steady calls with
# P ranks sharing the GPU at full Reddit shape (loaders' warm-up first)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
O=gpurun_out/${R06_OUT:-r06final}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for s in reddit pubmed rmat; do
  PMC_SHAPE=$s PMC_TAG=${R06_OUT:-r06final}/pmc_$s bash scripts/pmc_session.sh || { echo "PMC $s FAIL"; exit 1; }
done
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic'), d.get('first_call_seconds'), d.get('output_sha_ok'), {k: (round(v['ms_per_step'],4), round(v['roofline']['frac'],3), v.get('output_sha_ok')) for k,v in d.get('shapes',{}).items()}, d['classifier']['forward']['ms'], d['classifier']['backward']['ms'])"
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o p -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --shapes none > $R/$O/bench_prof.log 2>&1 || { tail $R/$O/bench_prof.log; exit 1; }
find $R/$O/prof -name "*kernel_stats.csv" -exec head -6 {} \; | cut -c1-160
cd $R
for P in 2 4 8; do
  mkdir -p $O/first_p$P
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$P \
     --master-addr=127.0.0.1 --master-port=$((29700+P)) tests/rank_precompute.py $O/first_p$P 232965 \
     > $O/first_p$P.log 2>&1 || { tail $O/first_p$P.log; exit 1; }
  cat $O/first_p$P/rank0.json; echo
done
