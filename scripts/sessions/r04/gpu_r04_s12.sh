set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# transposed quads (row_quadsT_pipe) for 33..64-float heavy rows: parity, then A/B vs pairs
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "narrow_launches" > $O/pytest_s12.log 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest_s12.log; exit 1; }
tail -2 $O/pytest_s12.log
timeout -k 10 300 python scripts/ab_tune.py --knob heavy_pairs --values 5,13 --widths 64,48,40 --rounds 8 > $O/quadsT_ab.log 2>&1 || { tail $O/quadsT_ab.log; exit 1; }
grep '^{' $O/quadsT_ab.log
