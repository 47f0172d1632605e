set -o pipefail
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "plan or ingest or tiny_cases_sgc or colsplit or column_groups" > $O/pytest_sort.log 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest_sort.log; exit 1; }
tail -3 $O/pytest_sort.log
for m in "" "--warm"; do for t in "" "--no-tiny"; do timeout -k 10 120 python scripts/first_call.py $m $t >> $O/first_call.log 2>&1 || exit 1; done; done
grep -v amdgpu $O/first_call.log
timeout -k 10 60 python scripts/micro/gather_cols.py /tmp/cols.bin > /dev/null && timeout -k 10 200 variants/gather_rate /tmp/cols.bin 10 64:64:0:0 64:64:0:32 64:64:0:64 76:96:0:0 76:96:0:32 76:80:0:20 80:80:0:0 96:96:0:0 96:96:0:32 12:16:0:0 16:16:0:0 32:32:0:0 48:48:0:0 128:128:0:0 > $O/gather_rate2.log 2>&1 || exit 1
grep -v amdgpu $O/gather_rate2.log | grep '"U": 4'
timeout -k 10 300 python -u scripts/ab_tune.py --kwarg threshold --values -1,22000 --widths 64,76,128 --rounds 8 > $O/thr.log 2>&1 || exit 1
grep -v amdgpu $O/thr.log
