"""Summarise a scripts/sweep_tune.sh directory: one line per run."""
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "*.json")), key=lambda p: int(os.path.basename(p)[:-5])):
    lines = [ln for ln in open(f).read().splitlines() if ln.startswith("{")]
    if not lines:
        print(os.path.basename(f), "no output")
        continue
    r = json.loads(lines[-1])
    rf = r.get("roofline", {})
    print(f"{os.path.basename(f):8s} {str(r.get('tuning', '-')):60s} step {r['ms_per_step']:.3f} "
          f"hop {rf.get('kernel_mean_ms', float('nan')):.3f} light "
          f"{rf.get('light_kernel_mean_ms') or float('nan'):.3f}")
    for k, v in r.get("shapes", {}).items():
        print(f"{'':8s} {k:60s} step {v['ms_per_step']:.3f} hop {v['roofline']['kernel_mean_ms']:.3f}")
