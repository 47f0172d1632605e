set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# hub threshold at the line partition's widths with the transposed heavy rows
timeout -k 10 400 python scripts/ab_tune.py --kwarg hub_threshold --values=-1,16384,8192,4096 --widths 64,128 --rounds 8 > $O/hubthr2.log 2>&1 || { tail $O/hubthr2.log; exit 1; }
grep '^{' $O/hubthr2.log
timeout -k 10 400 python scripts/ab_tune.py --kwarg threshold --values=-1,128,512,1024 --widths 64,128 --rounds 8 > $O/thr2.log 2>&1 || { tail $O/thr2.log; exit 1; }
grep '^{' $O/thr2.log
