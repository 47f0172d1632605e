set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# streaming classifier v4 (batched W staging): parity, timings incl. diag
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "linear_stream or linear_tile" > $O/pytest_s23.log 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest_s23.log; exit 1; }
tail -1 $O/pytest_s23.log
for lk in 2 4 3 1 2 4 3 1; do
  timeout -k 10 200 python -m sgc_amd.classifier_bench --tune linear_kernel=$lk > $O/cls5_lk$lk.log 2>&1 || { tail $O/cls5_lk$lk.log; exit 1; }
  grep -v amdgpu $O/cls5_lk$lk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lk=$lk', 'fwd', round(d['forward']['ms'],4))"
done
