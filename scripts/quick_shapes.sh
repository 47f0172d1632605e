#!/bin/bash
# Short single-GPU bench per shape, one summary line each (gpurun_out/shapes.log):
#   SHAPES="pubmed cora reddit" ARGS="--tune hub_stream=1" bash scripts/quick_shapes.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for sh in ${SHAPES:-pubmed cora reddit}; do
  timeout -k 10 300 python bench.py --shape "$sh" --shapes none --no-cpu-baseline \
      --steps "${STEPS_N:-30}" --warmup 5 ${ARGS} > gpurun_out/b_$sh.log 2>&1 || exit $?
  python - "$sh" "${ARGS}" >> gpurun_out/shapes.log <<'PY'
import json, sys
sh, args = sys.argv[1], sys.argv[2]
d = [json.loads(l) for l in open(f"gpurun_out/b_{sh}.log") if l.startswith("{")][0]
r = d["roofline"]
print(json.dumps({"shape": sh, "args": args, "G_edges_per_s": round(d["value"] / 1e9, 4),
                  "ms_per_step": round(d["ms_per_step"], 4), "hop_ms": round(r["kernel_mean_ms"], 4),
                  "light_ms": r["light_kernel_mean_ms"], "hub_ms": r["hub_kernel_mean_ms"],
                  "frac": r["frac"]}))
PY
done
cat gpurun_out/shapes.log
