set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# classifier v6 (dynamic per-CU tile grabbing): parity, timings incl. diag
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "linear or xent or autograd or fused or sgc_model" > $O/pytest_s26.log 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest_s26.log; exit 1; }
tail -1 $O/pytest_s26.log
for lk in 2 3 4 1 2 3 4 1; do
  timeout -k 10 200 python -m sgc_amd.classifier_bench --tune linear_kernel=$lk > $O/cls7_lk$lk.log 2>&1 || { tail $O/cls7_lk$lk.log; exit 1; }
  grep -v amdgpu $O/cls7_lk$lk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lk=$lk', 'fwd', round(d['forward']['ms'],4))"
done
