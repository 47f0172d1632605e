set -o pipefail
# round-4 final measurement: full GPU suite, smoke, PMC traffic records for
# the final library (Reddit, RMAT, Pubmed), bench N=1 and its rocprofv3
# kernel-trace summary, the two-rank self-launch.
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo PYTEST FAIL; grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
for s in reddit rmat pubmed; do
  PMC_SHAPE=$s PMC_TAG=r04f/pmc_$s bash scripts/pmc_session.sh || { echo "PMC $s FAIL"; exit 1; }
  cp profiles/pmc_$s.json $O/ 2>/dev/null
done
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('first_call_seconds'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --shapes "" --no-classifier > $GRAFT_REPO_ROOT/$O/bench_prof.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/bench_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline > $O/selfl.log 2>&1 || { tail $O/selfl.log; exit 1; }
grep '^{' $O/selfl.log | tail -1 | cut -c1-600
