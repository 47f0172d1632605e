set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# transposed pairs (heavy_pairs bit 16): parity, then A/B vs the untransposed pairs
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "narrow_launches" > $O/pytest_s13.log 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest_s13.log; exit 1; }
tail -2 $O/pytest_s13.log
timeout -k 10 400 python scripts/ab_tune.py --knob heavy_pairs --values 13,29 --widths 76,128,304,F --rounds 8 > $O/pairsT_ab.log 2>&1 || { tail $O/pairsT_ab.log; exit 1; }
grep '^{' $O/pairsT_ab.log
