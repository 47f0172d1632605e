set -o pipefail
# round-4 final, same library: PMC records, bench N=1 reading them, rocprofv3 stats of the bench, P = 2/4/8 rehearsals
O=gpurun_out/r04final2; mkdir -p $O
for s in reddit pubmed rmat; do
  PMC_SHAPE=$s PMC_TAG=r04final2/pmc_$s bash scripts/pmc_session.sh || { echo "PMC $s FAIL"; exit 1; }
done
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic'), d.get('first_call_seconds'), {k: (round(v['ms_per_step'],4), round(v['roofline']['frac'],3)) for k,v in d.get('shapes',{}).items()}, d['classifier']['forward']['ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --shapes none --no-classifier > $GRAFT_REPO_ROOT/$O/bench_prof.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/bench_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python scripts/line_rehearsal.py --P 8,4,2 --reps 8 > $O/line_rehearsal.log 2>&1 || { tail $O/line_rehearsal.log; exit 1; }
grep summary $O/line_rehearsal.log | cut -c1-420
timeout -k 10 500 python scripts/feature_rehearsal.py --P 8,4,2 --reps 8 > $O/feat_rehearsal.log 2>&1 || { tail $O/feat_rehearsal.log; exit 1; }
grep summary $O/feat_rehearsal.log | cut -c1-420
