#!/bin/bash
# CE kernels rows-in-flight A/B (variants/ce_r*.so, built from a scratch copy
# of csrc with the rows-in-flight loss.hip; the shipped library is the
# default): CE parity tests on the R=4 variant, per-library timings, then a
# kernel-trace profile of the R=4 variant and of the default library.
set -o pipefail
O=gpurun_out/ce
mkdir -p $O
SGC_AMD_LIB=variants/ce_r4.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q \
    --timeout 120 --timeout-method thread -k "entropy or logits or closure" > $O/pytest.log 2>&1 || exit 1
for lib in default variants/ce_r1.so variants/ce_r2.so variants/ce_r4.so variants/ce_r8.so default; do
    if [ $lib = default ]; then
        timeout -k 10 120 python -u scripts/ce_ab.py >> $O/ab.log 2>&1 || exit 1
    else
        SGC_AMD_LIB=$lib timeout -k 10 120 python -u scripts/ce_ab.py >> $O/ab.log 2>&1 || exit 1
    fi
done
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_default -o run -- python3 scripts/ce_ab.py > $O/prof_default.log 2>&1 || exit 1
SGC_AMD_LIB=variants/ce_r4.so timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof_r4 -o run -- python3 scripts/ce_ab.py > $O/prof_r4.log 2>&1
