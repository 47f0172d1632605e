set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# streaming classifier forward: parity (forced and auto), then A/B vs the LDS tile
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "linear or xent or autograd or fused or sgc_model" > $O/pytest_s17.log 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest_s17.log; exit 1; }
tail -2 $O/pytest_s17.log
for lk in 2 1 2 1; do
  timeout -k 10 200 python -m sgc_amd.classifier_bench --tune linear_kernel=$lk > $O/classifier_lk$lk.log 2>&1 || { tail $O/classifier_lk$lk.log; exit 1; }
  grep -v amdgpu $O/classifier_lk$lk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lk=$lk', 'fwd', round(d['forward']['ms'],4), 'frac', round(d['forward']['frac'],3), 'bwd', round(d['backward']['ms'],4), 'closure', round(d['closure']['dropin_ms'],4), 'lbfgs', round(d['lbfgs']['dropin_ms'],2))"
done
