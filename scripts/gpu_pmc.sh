#!/bin/bash
# rocprofv3 PMC passes for the SpMM's HBM traffic (one counter set per pass,
# kernel trace only beside the counters) -> profiles/pmc_reddit.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$(pwd); OUT=$R/gpurun_out; mkdir -p "$OUT"
export PMC_META=$OUT/pmc_meta${SGC_PMC_TAG}.json
cd /tmp && export TMPDIR=/tmp
for pass in "fetch:FETCH_SIZE" "write:WRITE_SIZE" "l2:TCC_HIT_sum TCC_MISS_sum"; do
  name=${pass%%:*}; ctr=${pass#*:}
  d="$OUT/pmc_${name}${SGC_PMC_TAG}"; rm -rf "$d"
  timeout -k 10 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d "$d" -o p \
     -- python3 "$R/scripts/pmc_traffic.py" workload > "$d.log" 2>&1
  rc=$?; echo "[pmc $name$SGC_PMC_TAG] rc=$rc"; grep "pmc workload" "$d.log"
  [ $rc -ne 0 ] && exit $rc
done
cd "$R" && python3 scripts/pmc_traffic.py summarize "$OUT" > "$OUT/pmc_summary$SGC_PMC_TAG.log" 2>&1; echo "[summary] rc=$?"; grep -E "hbm_bytes_per_launch|l2_hit|traffic_over" "$OUT/pmc_summary$SGC_PMC_TAG.log"
