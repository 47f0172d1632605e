#!/bin/bash
# Hub workgroup size (15 vs 7 loader waves): parity, N=1 Reddit, P=8 rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
    --timeout-method thread -k "long_hub or hub_stream or schedule" > gpurun_out/pt.log 2>&1
rc=$?; tail -1 gpurun_out/pt.log; [ $rc -eq 0 ] || exit $rc
for a in "" "--tune hub_loaders=7"; do
  SHAPES="reddit" ARGS="$a" bash scripts/quick_shapes.sh > /dev/null || exit $?
done
cat gpurun_out/shapes.log
timeout -k 10 400 python scripts/cyclic_rehearsal.py --P 8 --groups 1,2,3 --tune hub_loaders=7 \
    > gpurun_out/cyc7.log 2>&1 || exit $?
grep summary gpurun_out/cyc7.log | cut -c1-300
