set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# line partition: per-rank rehearsal (P = 2/4/8) beside the feature partition, then full-size P=8 bit-exactness
timeout -k 10 400 python scripts/line_rehearsal.py --P 8,4,2 --reps 8 > $O/line_rehearsal.log 2>&1 || { tail $O/line_rehearsal.log; exit 1; }
grep summary $O/line_rehearsal.log
timeout -k 10 400 python scripts/feature_rehearsal.py --P 8,4 --exchange alltoall --reps 8 > $O/feat_rehearsal.log 2>&1 || { tail $O/feat_rehearsal.log; exit 1; }
grep summary $O/feat_rehearsal.log | cut -c1-400
timeout -k 10 600 python -u -m pytest tests/test_gpu_multigpu.py -x -q --timeout 580 --timeout-method thread -k "p8_partition_full_size and lines" > $O/pytest_lines_p8.log 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest_lines_p8.log; exit 1; }
tail -2 $O/pytest_lines_p8.log
