# round-4 session 3: the narrow pass's tail (hub threshold / heavy rows),
# Pubmed with no hub kernel, LBFGS timing
set -o pipefail
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 300 python -u scripts/narrow_pass.py --widths 64,76,128 --reps 10 > $O/narrow_pass.log 2>&1 || { tail $O/narrow_pass.log; exit 1; }
grep -v amdgpu $O/narrow_pass.log
timeout -k 10 400 python -u scripts/ab_tune.py --kwarg hub_threshold --values=-1,8192,4096,2048,1024 --widths 64,76,128 --rounds 6 > $O/hubthr.log 2>&1 || { tail $O/hubthr.log; exit 1; }
grep -v amdgpu $O/hubthr.log
timeout -k 10 300 python -u scripts/ab_tune.py --kwarg hub_threshold --values=-1,100000 --shape pubmed --widths 500 --rounds 20 > $O/pubmed_hub.log 2>&1 || { tail $O/pubmed_hub.log; exit 1; }
grep -v amdgpu $O/pubmed_hub.log
timeout -k 10 200 python -m sgc_amd.classifier_bench > $O/classifier2.log 2>&1 || { tail $O/classifier2.log; exit 1; }
grep -v amdgpu $O/classifier2.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_multigpu.py -x -q --timeout 200 --timeout-method thread -k "mgpu or device_set" > $O/pytest_mgpu.log 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest_mgpu.log; exit 1; }
tail -3 $O/pytest_mgpu.log
