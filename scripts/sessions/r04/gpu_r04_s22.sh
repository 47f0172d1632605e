set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# streaming classifier v3 (scalar wave index -> scalar tile/chunk control): parity, timings, diag, counters
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "linear or xent or autograd or fused or sgc_model" > $O/pytest_s22.log 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest_s22.log; exit 1; }
tail -1 $O/pytest_s22.log
for lk in 2 1 3 4 2 1; do
  timeout -k 10 200 python -m sgc_amd.classifier_bench --tune linear_kernel=$lk > $O/cls4_lk$lk.log 2>&1 || { tail $O/cls4_lk$lk.log; exit 1; }
  grep -v amdgpu $O/cls4_lk$lk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lk=$lk', 'fwd', round(d['forward']['ms'],4), 'closure', round(d['closure']['dropin_ms'],4))"
done
bash scripts/pmc_classifier.sh > $O/pmc_cls7.log 2>&1 || { cat $O/pmc_cls7.log; exit 1; }
cat gpurun_out/pmc_cls/sq.summary gpurun_out/pmc_cls/insts.summary gpurun_out/pmc_cls/lds.summary | grep -E 'linear_stream'
