set -o pipefail
O=gpurun_out/r04s16; mkdir -p $O
# full GPU suite on the library with transposed heavy rows + the line partition; smoke; 4-rank gloo bench (lines behind the public call)
timeout -k 10 1000 python -u -m pytest tests -q -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo PYTEST FAIL; grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 500 python bench.py --gpus 4 --dist-backend gloo --steps 3 --warmup 1 --no-cpu-baseline > $O/bench4.log 2>&1 || { tail $O/bench4.log; exit 1; }
grep '^{' $O/bench4.log | tail -1 | cut -c1-1500
