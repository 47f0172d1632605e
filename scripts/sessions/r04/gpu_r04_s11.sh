set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# heavy threshold at narrow widths: heavy rows through the light path (length order) vs the pairs path
timeout -k 10 300 python scripts/ab_tune.py --kwarg threshold --values=-1,512,2048,16384 --widths 64,76,128 --rounds 6 > $O/thr_narrow.log 2>&1 || { tail $O/thr_narrow.log; exit 1; }
grep '^{' $O/thr_narrow.log
timeout -k 10 300 python scripts/ab_tune.py --knob heavy_pairs --values 5,4,0 --widths 64,76 --rounds 6 > $O/pairs_narrow.log 2>&1 || { tail $O/pairs_narrow.log; exit 1; }
grep '^{' $O/pairs_narrow.log
