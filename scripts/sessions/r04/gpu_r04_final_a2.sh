set -o pipefail
# round-4 final (a, continued): the fixed timing test, smoke, bench N=1 and its rocprofv3 kernel-trace summary
O=gpurun_out/r04final; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "timing_hooks" > $O/pytest_timing.log 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest_timing.log; exit 1; }
tail -1 $O/pytest_timing.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('first_call_seconds'), {k: round(v['ms_per_step'],4) for k,v in d.get('shapes',{}).items()}, d['classifier']['forward']['ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --shapes none --no-classifier > $GRAFT_REPO_ROOT/$O/bench_prof.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/bench_prof.log; exit 1; }
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" -exec head -5 {} \; | cut -c1-220
