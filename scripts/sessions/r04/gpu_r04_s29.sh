set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# column groups at the line partition's widths (64 / 96 / 128 floats, all rows): is the L2 share worth a partial-sum pass?
timeout -k 10 400 python scripts/ab_tune.py --attr COLUMN_GROUPS --values 1,2,3 --widths 64,96,128 --rounds 8 > $O/groups_narrow.log 2>&1 || { tail $O/groups_narrow.log; exit 1; }
grep '^{' $O/groups_narrow.log
