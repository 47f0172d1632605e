set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# round-4 session 7: classifier kernels v2 (double-buffered LDS tile, deeper dW prefetch)
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "linear or xent or autograd or fused or prepared or graphed or layouts or schedule" > $O/pytest_s7.log 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest_s7.log; exit 1; }
tail -2 $O/pytest_s7.log
timeout -k 10 200 python -m sgc_amd.classifier_bench > $O/classifier3.log 2>&1 || { tail $O/classifier3.log; exit 1; }
grep -v amdgpu $O/classifier3.log
bash scripts/pmc_classifier.sh > $O/pmc_cls2.log 2>&1 || { cat $O/pmc_cls2.log; exit 1; }
cat gpurun_out/pmc_cls/sq.summary gpurun_out/pmc_cls/insts.summary | grep -E '"linear_kernel"|"kernel": ""'
# round-4 session 8: the hub kernel's share of a narrow pass (knobs), bench N=1 full line
timeout -k 10 300 python -u scripts/ab_tune.py --knob hub_loaders --values 15,7 --widths 76,152,304 --rounds 8 > $O/hubload_ab.log 2>&1 || { tail $O/hubload_ab.log; exit 1; }
grep -v amdgpu $O/hubload_ab.log
timeout -k 10 300 python -u scripts/ab_tune.py --knob hub_chunk --values 0,64 --widths 76 --rounds 8 > $O/hubchunk_ab.log 2>&1 || { tail $O/hubchunk_ab.log; exit 1; }
grep -v amdgpu $O/hubchunk_ab.log

timeout -k 10 200 python -u scripts/host_overhead.py > $O/hostov.log 2>&1 || { tail $O/hostov.log; exit 1; }
grep -v amdgpu $O/hostov.log

timeout -k 10 300 python -u scripts/ab_tune.py --kwarg hub_threshold --values=-1,512,1000 --shape pubmed --widths 500 --rounds 20 > $O/pubmed_hub2.log 2>&1 || { tail $O/pubmed_hub2.log; exit 1; }
grep -v amdgpu $O/pubmed_hub2.log
