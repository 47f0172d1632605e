set -o pipefail
# round-4 final (b): PMC traffic records for this library (Reddit, RMAT, Pubmed), then bench N=1 reading them, 2-rank self-launch
O=gpurun_out/r04final; mkdir -p $O
for s in reddit pubmed rmat; do
  PMC_SHAPE=$s PMC_TAG=r04final/pmc_$s bash scripts/pmc_session.sh || { echo "PMC $s FAIL"; exit 1; }
done
timeout -k 10 600 python bench.py > $O/bench2.log 2>&1 || { tail $O/bench2.log; exit 1; }
grep '^{' $O/bench2.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('traffic'), d.get('first_call_seconds'), {k: (round(v['ms_per_step'],4), round(v['roofline']['frac'],3)) for k,v in d.get('shapes',{}).items()})"
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline > $O/selfl.log 2>&1 || { tail $O/selfl.log; exit 1; }
grep '^{' $O/selfl.log | tail -1 | cut -c1-400
