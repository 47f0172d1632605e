set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# classifier v8: two 16-row m-tiles per wave (8-wave workgroups): parity, timings (mt 2 vs 1, diag)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "linear or xent or autograd or fused or sgc_model" > $O/pytest_s32.log 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest_s32.log; exit 1; }
tail -1 $O/pytest_s32.log
for cfg in "linear_mt=2" "linear_mt=1" "linear_kernel=1" "linear_mt=2" "linear_mt=1" "linear_kernel=1"; do
  timeout -k 10 200 python -m sgc_amd.classifier_bench --tune $cfg > $O/cls9.log 2>&1 || { tail $O/cls9.log; exit 1; }
  grep -v amdgpu $O/cls9.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', 'fwd', round(d['forward']['ms'],4))"
done
