# round-4 session 8: the hub kernel's share of a narrow pass (knobs), bench N=1 full line
set -o pipefail
O=gpurun_out/r04; mkdir -p $O
timeout -k 10 300 python -u scripts/ab_tune.py --knob hub_loaders --values 15,7 --widths 76,152,304 --rounds 8 > $O/hubload_ab.log 2>&1 || { tail $O/hubload_ab.log; exit 1; }
grep -v amdgpu $O/hubload_ab.log
timeout -k 10 300 python -u scripts/ab_tune.py --knob hub_chunk --values 0,64 --widths 76 --rounds 8 > $O/hubchunk_ab.log 2>&1 || { tail $O/hubchunk_ab.log; exit 1; }
grep -v amdgpu $O/hubchunk_ab.log
