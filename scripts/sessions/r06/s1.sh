#!/bin/bash
# round 6 session 1: the new parity tests (public call at full size, IPC
# exchange at world 1 and with ranks sharing the GPU, first-call partitions)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}" || exit 2
O=gpurun_out/r06_s1${TAG:-}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -x -v --timeout-method thread -m gpu"
timeout -k 10 300 $T --timeout 280 tests/test_gpu_multigpu.py -k "rccl_exchange_paths_world1" > $O/t1.log 2>&1 &&
timeout -k 10 600 $T --timeout 280 tests/test_gpu_multigpu.py -k "under_torchrun_matches_one_gpu or auto_first_call" > $O/t2.log 2>&1 &&
timeout -k 10 900 $T --timeout 880 tests/test_gpu_multigpu.py -k "test_p8_partition_full_size_bit_exact and reddit and (lines or features)" > $O/t3.log 2>&1 &&
timeout -k 10 600 $T --timeout 580 tests/test_gpu_parity.py -k "public_call or shape_hash" > $O/t4.log 2>&1
rc=$?
echo "rc=$rc"
tail -5 $O/t*.log
exit $rc
