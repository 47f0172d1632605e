#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; a fault-like exit (anything but 0/1:
# timeout 124/137, abort 134, segfault 139) stops the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
ROOTDIR=$(pwd)
OUT=$ROOTDIR/gpurun_out
mkdir -p "$OUT"
STEPS=${STEPS:-"pytest smoke bench prof"}
# progress marker for long single steps (the RMAT-shape test and bench leg
# each run a few minutes without a new output line)
( while sleep 45; do date +%T >> "$OUT/heartbeat.log"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() {
  local name=$1; shift
  local t0=$(date +%s)
  "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$name] rc=$rc $(( $(date +%s) - t0 ))s"
  tail -5 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fault-like exit from $name; stopping"; exit $rc; fi
  return 0
}
for s in $STEPS; do
  case $s in
    pytest) run pytest timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS} ;;
    cyc)    run cyc timeout -k 10 900 python scripts/cyclic_rehearsal.py ${CYC_ARGS} ;;
    feat)   run feat timeout -k 10 400 python scripts/feature_rehearsal.py ${FEAT_ARGS} ;;
    p8)     run p8 timeout -k 10 600 python scripts/p8_rehearsal.py ${P8_ARGS} ;;
    rankwork) run rankwork timeout -k 10 400 python scripts/rank_work.py ;;
    smoke)  run smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench timeout -k 10 600 python bench.py ${BENCH_ARGS} ;;
    aux)    run aux timeout -k 10 600 python scripts/bench_aux.py ;;
    hostov) run hostov timeout -k 10 300 python scripts/host_overhead.py ;;
    ab2)    run ab2 timeout -k 10 400 python scripts/ab_tune.py ${AB2_ARGS} ;;
    narrow) run narrow timeout -k 10 300 python scripts/narrow_pass.py ${NARROW_ARGS} ;;
    ab)     run ab timeout -k 10 400 python scripts/ab_tune.py ${AB_ARGS} ;;
    ab8)    run ab8 timeout -k 10 300 python scripts/ab_tune.py --widths F --rows 8:0 ${AB8_ARGS:-$AB_ARGS} ;;
    locality) run locality timeout -k 10 400 python scripts/locality_ab.py ${LOCALITY_ARGS} ;;
    selfl)  run selfl timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 3 \
                --warmup 1 --no-cpu-baseline ${DIST_ARGS} ;;
    rccl1)  run rccl1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
                --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 1 --steps 5 --warmup 2 \
                --distributed-path --no-cpu-baseline ${DIST_ARGS} ;;
    dist)   run dist timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
                --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
                --dist-backend gloo ${DIST_ARGS} ;;
    dcheck) # 8 ranks on the one GPU (gloo, host-staged exchange): bit-exact X_K at full size
            IFS=, read -ra VARIANTS <<< "${DCHECK_VARIANTS:---partition rows,--partition rows --row-chunks 4,--partition rows --group-floats 256,--partition tiles --col-blocks 2,--partition tiles --col-blocks 4}"
            for v in "${VARIANTS[@]}"; do
              run dcheck timeout -k 10 ${DCHECK_TIMEOUT:-400} python -m torch.distributed.run --nnodes=1 \
                  --nproc-per-node ${DCHECK_RANKS:-8} --master-addr 127.0.0.1 --master-port 29537 \
                  scripts/dist_check.py --shape ${DCHECK_SHAPE:-reddit} $v --cache "${TMPDIR:-/tmp}"
              grep -h '^{' "$OUT/dcheck.log" >> "$OUT/dcheck_all.log"
            done ;;
    rdist)  run rdist timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
                --master-addr 127.0.0.1 --master-port 29536 drivers/reddit_dist.py --check --test ;;
    ndiag)  run ndiag bash "$ROOTDIR/scripts/narrow_diag.sh" ;;
    pmc)    for sh in ${PMC_SHAPES:-reddit rmat}; do
              run pmc_$sh env PMC_SHAPE=$sh bash "$ROOTDIR/scripts/pmc_session.sh"
            done ;;
    prof)   cd /tmp && export TMPDIR=/tmp && \
            run prof timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run \
                --output-format csv -- python3 "$ROOTDIR/bench.py" --steps 10 --warmup 3 --no-cpu-baseline \
                --shapes none ${BENCH_ARGS}
            cd "$ROOTDIR" ;;
  esac
done
