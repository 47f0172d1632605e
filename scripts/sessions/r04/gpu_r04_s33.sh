set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# classifier v9: 64-k chunks (two deep): parity, timings (ck 64 vs 32, diag at 64)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "linear or xent or autograd or fused or sgc_model" > $O/pytest_s33.log 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest_s33.log; exit 1; }
tail -1 $O/pytest_s33.log
for cfg in "linear_ck=64" "linear_ck=32" "linear_ck=64" "linear_ck=32"; do
  timeout -k 10 200 python -m sgc_amd.classifier_bench --tune $cfg > $O/cls10.log 2>&1 || { tail $O/cls10.log; exit 1; }
  grep -v amdgpu $O/cls10.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', 'fwd', round(d['forward']['ms'],4))"
done
