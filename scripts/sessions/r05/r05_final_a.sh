set -o pipefail
# round-5 final: full GPU suite, smoke
O=gpurun_out/${R05_OUT:-r05final}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo PYTEST FAIL; grep -E "FAILED|Error" $O/pytest.log | head -20; tail -5 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
