set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# line partition with the tail on its own stream (+ per-caller-stream hub side streams)
timeout -k 10 400 python scripts/line_rehearsal.py --P 8,4 --reps 8 > $O/line_rehearsal2.log 2>&1 || { tail $O/line_rehearsal2.log; exit 1; }
grep summary $O/line_rehearsal2.log | cut -c1-330
timeout -k 10 600 python -u -m pytest tests/test_gpu_multigpu.py -x -q --timeout 580 --timeout-method thread -k "p8_partition_full_size and lines" > $O/pytest_lines_p8b.log 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest_lines_p8b.log; exit 1; }
tail -1 $O/pytest_lines_p8b.log
