#!/bin/bash
# Schedule-knob sweep: one bench.py run per combination in $COMBOS (each a
# comma list of KEY=VALUE for --tune; "-" = defaults), no CPU baseline, each
# under its own time limit; JSON lines into gpurun_out/sweep/<i>.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out/${SWEEP_TAG:-sweep}
mkdir -p $OUT
i=0
for combo in ${COMBOS:--}; do
  args=""
  if [ "$combo" != "-" ]; then
    for kv in ${combo//,/ }; do args="$args --tune $kv"; done
  fi
  timeout -k 10 300 python bench.py --steps ${STEPS_N:-10} --warmup 3 --no-cpu-baseline \
    --shapes ${SHAPES:-none} ${EXTRA} $args > $OUT/$i.json 2> $OUT/$i.err
  rc=$?
  echo "[$i] $combo rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  i=$((i+1))
done
exit 0
