# round-4 session 2: sort/ingest/plan + classifier tests, first-call, classifier
# timing, gather-shape sweep, heavy-threshold A/B (each step time-limited)
set -o pipefail
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multigpu.py::test_mgpu_handles_survive_reinit tests/test_gpu_multigpu.py::test_mgpu_engine_virtual_devices_bit_exact tests/test_gpu_multigpu.py::test_mgpu_engine_reddit_shape_hash -x -q --timeout 120 --timeout-method thread -k "plan or ingest or tiny_cases_sgc or colsplit or column_groups or linear or xent or autograd or fused or native" > $O/pytest_s2.log 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest_s2.log; exit 1; }
tail -3 $O/pytest_s2.log
for m in "" "--warm"; do for t in "" "--no-tiny"; do timeout -k 10 120 python scripts/first_call.py $m $t >> $O/first_call.log 2>&1 || exit 1; done; done
grep -v amdgpu $O/first_call.log
timeout -k 10 200 python -m sgc_amd.classifier_bench > $O/classifier.log 2>&1 || { tail $O/classifier.log; exit 1; }
grep -v amdgpu $O/classifier.log
timeout -k 10 60 python scripts/micro/gather_cols.py /tmp/cols.bin > /dev/null && timeout -k 10 200 variants/gather_rate /tmp/cols.bin 10 64:64:0:0 64:64:0:32 64:64:0:64 76:96:0:0 76:96:0:32 76:80:0:20 80:80:0:0 96:96:0:0 96:96:0:32 12:16:0:0 16:16:0:0 32:32:0:0 48:48:0:0 128:128:0:0 > $O/gather_rate2.log 2>&1 || exit 1
grep -v amdgpu $O/gather_rate2.log | grep '"U": 4'
timeout -k 10 300 python -u scripts/ab_tune.py --kwarg threshold --values -1,22000 --widths 64,76,128 --rounds 8 > $O/thr.log 2>&1 || exit 1
grep -v amdgpu $O/thr.log
