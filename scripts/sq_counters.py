"""Where the SpMM kernels' waves spend their cycles (rocprofv3 SQ counters).

    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \\
        SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAVES \\
        --kernel-trace --output-format csv -d OUT -o p -- python3 scripts/pmc_traffic.py workload reddit
    python scripts/sq_counters.py OUT

Per kernel: the mean of each counter per dispatch and the shares of
SQ_WAVE_CYCLES (MI355X_MICROARCH.md, rocprofv3 PMC slots: WAIT_ANY = waves
parked on s_waitcnt / barriers, WAIT_INST_ANY = issue stalls, ACTIVE_INST_ANY
= issuing; the three are disjoint and sum to about WAVE_CYCLES).  One JSON
line per kernel.
"""
import collections
import csv
import glob
import json
import os
import sys


def kernel_label(name):
    """'void sgc::(anonymous namespace)::xent_dw_kernel<2, 3, 2>(float const*, ...)'
    -> 'xent_dw_kernel<2, 3, 2>' (the anonymous namespace's parentheses must
    go before the argument list is cut: round 5's summaries cut at them and
    labelled every kernel '')."""
    k = name.replace("(anonymous namespace)::", "").replace("void ", "")
    depth, cut = 0, len(k)
    for i, ch in enumerate(k):  # the first '(' outside the template arguments
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    return k[:cut].split("::")[-1].strip() if "::" in k[:cut].split("<")[0] else k[:cut].strip()


def main(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                k = kernel_label(r.get("Kernel_Name", ""))
                did = r.get("Dispatch_Id", r.get("Correlation_Id", ""))
                per[k][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[k].add(did)
    for k, c in sorted(per.items()):
        n = max(1, len(disp[k]))
        mean = {name: v / n for name, v in c.items()}
        wc = mean.get("SQ_WAVE_CYCLES", 0.0)
        shares = {}
        if wc:
            for name in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                         "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS"):
                if name in mean:
                    shares[name] = round(mean[name] / wc, 4)
        print(json.dumps({"kernel": k, "dispatches": n,
                          "per_dispatch": {a: round(b, 1) for a, b in mean.items()},
                          "share_of_wave_cycles": shares}))


if __name__ == "__main__":
    main(sys.argv[1])
