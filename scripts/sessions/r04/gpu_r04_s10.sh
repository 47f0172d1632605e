set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# round-4 session 10: classifier tile v3 (buffer loads, hoisted offsets, aligned b128 operand reads), 1 vs 2 LDS images
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "linear or xent or autograd or fused or prepared or tile" > $O/pytest_s10.log 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest_s10.log; exit 1; }
tail -2 $O/pytest_s10.log
for nb in 2 1 2 1; do
  timeout -k 10 200 python -m sgc_amd.classifier_bench --tune tile_buffers=$nb > $O/classifier_v3_nb$nb.log 2>&1 || { tail $O/classifier_v3_nb$nb.log; exit 1; }
  grep -v amdgpu $O/classifier_v3_nb$nb.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('nb=$nb', 'fwd', round(d['forward']['ms'],4), 'bwd', round(d['backward']['ms'],4), 'closure', round(d['closure']['dropin_ms'],4), 'fused', round(d['closure']['fused_sgc_cross_entropy_ms'],4), 'lbfgs', round(d['lbfgs']['dropin_ms'],2))"
done
bash scripts/pmc_classifier.sh > $O/pmc_cls3.log 2>&1 || { cat $O/pmc_cls3.log; exit 1; }
cat gpurun_out/pmc_cls/sq.summary gpurun_out/pmc_cls/insts.summary gpurun_out/pmc_cls/lds.summary | grep -E '"linear_kernel"|"kernel": ""'
