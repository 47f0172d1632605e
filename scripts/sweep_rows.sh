#!/bin/bash
# Light-kernel variants (rows_per_wave 1/2/4) on every BASELINE shape, one
# bench.py run each (no CPU baseline), under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/sweep_rows
mkdir -p $OUT
for rpw in ${RPW:-2 1 4}; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --shapes ${SHAPES:-pubmed,rmat} \
    --tune rows_per_wave=$rpw ${EXTRA} > $OUT/rpw$rpw.json 2> $OUT/rpw$rpw.err
  rc=$?
  echo "rows_per_wave=$rpw rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
