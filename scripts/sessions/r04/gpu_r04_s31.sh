set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# the line partition's tail launch (96 floats over a P = 8 rank's 1/8 nnz-balanced rows): hub / heavy thresholds
for r in 0 3; do
timeout -k 10 300 python scripts/ab_tune.py --rows 8:$r --kwarg hub_threshold --values=-1,1024,8192,30000 --widths 96 --rounds 10 > $O/tail_hubthr_r$r.log 2>&1 || { tail $O/tail_hubthr_r$r.log; exit 1; }
grep '^{' $O/tail_hubthr_r$r.log
timeout -k 10 300 python scripts/ab_tune.py --rows 8:$r --kwarg threshold --values=-1,64,256,1024 --widths 96 --rounds 10 > $O/tail_thr_r$r.log 2>&1 || { tail $O/tail_thr_r$r.log; exit 1; }
grep '^{' $O/tail_thr_r$r.log
done
