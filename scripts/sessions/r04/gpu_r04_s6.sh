# round-4 session 6: classifier counters, bench N=1 quick line (first call),
# bench --gpus 2 gloo test, mgpu + native-groups tests
set -o pipefail
O=gpurun_out/r04; mkdir -p $O
bash scripts/pmc_classifier.sh > $O/pmc_cls.log 2>&1 || { cat $O/pmc_cls.log; exit 1; }
cat gpurun_out/pmc_cls/*.summary | grep -E "linear_kernel|xent_dw|xent_reduce"
timeout -k 10 300 python -u -m pytest tests/test_gpu_multigpu.py tests/test_gpu_parity.py -x -q --timeout 280 --timeout-method thread -k "mgpu or device_set or bench_self_launch or column_groups_medium or native or narrow" > $O/pytest_s6.log 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest_s6.log; exit 1; }
tail -3 $O/pytest_s6.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --shapes none --no-cpu-baseline > $O/bench_quick.log 2>&1 || { tail $O/bench_quick.log; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_quick.log').read().strip().splitlines()[-1]);print({k:d[k] for k in ('value','ms_per_step','first_call_seconds','loader_warmup_seconds')}, d['roofline']['frac'])"
