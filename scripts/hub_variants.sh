#!/bin/bash
# Hub-kernel variants: the largest hub row alone (scripts/hub_probe.py), then
# the Reddit K=2 bench, per library build under variants/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
OUT=gpurun_out; mkdir -p $OUT
for v in ${VARIANTS:-pre3 pre4 pre8 nochain noload}; do
  SGC_AMD_LIB=variants/$v.so HUB_PROBE_WIDTHS=${WIDTHS:-602} HUB_PROBE_MODES=hub64,hub32 \
    timeout -k 10 120 python scripts/hub_probe.py >> $OUT/hub_variants.log 2>&1 || exit $?
done
for v in ${BENCH_VARIANTS:-pre3 pre4 pre8}; do
  echo "== $v" >> $OUT/hub_variants_bench.log
  SGC_AMD_LIB=variants/$v.so timeout -k 10 180 python bench.py --no-cpu-baseline --steps 20 \
    >> $OUT/hub_variants_bench.log 2>&1 || exit $?
done
