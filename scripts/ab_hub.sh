#!/bin/bash
# Interleaved A/B of where the hub kernel runs (hub_stream 0: hub on a side
# stream, light on the caller's; 3: hub on the caller's stream, light on the
# side stream) at the full Reddit shape, the 76-float pass and rank 0 of 8.
set -o pipefail
O=gpurun_out/ab_hub; mkdir -p $O
ab() { local name=$1; shift; timeout -k 10 300 python scripts/ab_tune.py "$@" > $O/$name.log 2>&1; local rc=$?; grep '^{' $O/$name.log; return $rc; }
ab stream3 --knob hub_stream --values 0,3 --widths F,76 --rounds 10 &&
ab stream3_p8 --knob hub_stream --values 0,3 --widths F,76 --rows 8:0 --rounds 10 &&
ab stream3_rmat --knob hub_stream --values 0,3 --shape rmat --widths F --rounds 3
