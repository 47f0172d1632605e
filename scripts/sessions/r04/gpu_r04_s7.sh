# round-4 session 7: classifier kernels v2 (double-buffered LDS tile, deeper dW prefetch)
set -o pipefail
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "linear or xent or autograd or fused" > $O/pytest_s7.log 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest_s7.log; exit 1; }
tail -2 $O/pytest_s7.log
timeout -k 10 200 python -m sgc_amd.classifier_bench > $O/classifier3.log 2>&1 || { tail $O/classifier3.log; exit 1; }
grep -v amdgpu $O/classifier3.log
bash scripts/pmc_classifier.sh > $O/pmc_cls2.log 2>&1 || { cat $O/pmc_cls2.log; exit 1; }
cat gpurun_out/pmc_cls/sq.summary gpurun_out/pmc_cls/insts.summary | grep -E '"linear_kernel"|"kernel": ""'
