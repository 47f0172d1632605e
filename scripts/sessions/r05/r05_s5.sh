set -o pipefail
# round-5 session 5: recorded launch lists (sgc_launch_list_*): full GPU suite,
# Pubmed host breakdown, bench N=1 (all shapes)
O=gpurun_out/r05s5; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo PYTEST FAIL; grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python scripts/host_breakdown.py > $O/host_breakdown.log 2>&1 || { tail $O/host_breakdown.log; exit 1; }
tail -1 $O/host_breakdown.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], {k: (round(v['ms_per_step'],4), round(v['roofline']['frac'],3)) for k,v in d.get('shapes',{}).items()}, d['classifier']['forward']['ms'], d['classifier']['forward'].get('single_call_ms'))"
