set -o pipefail
# round-5 final: PMC records, bench N=1 reading them, rocprofv3 stats of the bench
O=gpurun_out/${R05_OUT:-r05final}; mkdir -p $O
for s in reddit pubmed rmat; do
  PMC_SHAPE=$s PMC_TAG=${R05_OUT:-r05final}/pmc_$s bash scripts/pmc_session.sh || { echo "PMC $s FAIL"; exit 1; }
done
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic'), d.get('first_call_seconds'), {k: (round(v['ms_per_step'],4), round(v['roofline']['frac'],3)) for k,v in d.get('shapes',{}).items()}, d['classifier']['forward']['ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --shapes none > $GRAFT_REPO_ROOT/$O/bench_prof.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/bench_prof.log; exit 1; }
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" -exec head -4 {} \; | cut -c1-160
