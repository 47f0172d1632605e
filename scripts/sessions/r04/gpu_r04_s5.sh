# round-4 session 5: quads heavy path (narrow launches) -- parity, then A/B
set -o pipefail
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "narrow or accumulate or heavy_split or tiny_cases_sgc or reddit_shape_hash" > $O/pytest_s5.log 2>&1 || { echo PYTEST FAIL; tail -30 $O/pytest_s5.log; exit 1; }
tail -3 $O/pytest_s5.log
timeout -k 10 400 python -u scripts/ab_tune.py --knob heavy_pairs --values 1,5 --widths 64,32,16,12,48 --rounds 8 > $O/quads_ab.log 2>&1 || { tail $O/quads_ab.log; exit 1; }
grep -v amdgpu $O/quads_ab.log
timeout -k 10 300 python -u scripts/tail_probe.py --widths 64,32,12 > $O/tail_probe2.log 2>&1 || exit 1
grep -v amdgpu $O/tail_probe2.log
timeout -k 10 400 python -u scripts/ab_tune.py --knob rows_per_wave --values 0,4 --widths F,602,304,128 --rounds 6 > $O/rpw4_ab.log 2>&1 || { tail $O/rpw4_ab.log; exit 1; }
grep -v amdgpu $O/rpw4_ab.log
