#!/bin/bash
# Interleaved A/B of the pipeline-schedule knobs (light_pipe, pairs_pipe,
# chunks_pipe): each value's output checked bit-identical to the other's.
set -o pipefail
O=gpurun_out/ab1; mkdir -p $O
ab() { local name=$1; shift; timeout -k 10 300 python scripts/ab_tune.py "$@" > $O/$name.log 2>&1; local rc=$?; grep '^{' $O/$name.log; return $rc; }
ab light --knob light_pipe --values 0,1 --widths F,76,128,64 --rounds 8 &&
ab pairs --knob pairs_pipe --values 0,1 --widths F,76 --rounds 8 &&
ab light_p8 --knob light_pipe --values 0,1 --widths F,76 --rows 8:0 --rounds 8 &&
ab chunks_pubmed --knob chunks_pipe --values 0,1 --shape pubmed --widths F --rounds 10 &&
ab chunks_rmat --knob chunks_pipe --values 0,1 --shape rmat --widths F --rounds 3
