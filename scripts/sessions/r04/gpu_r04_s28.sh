set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# fused hub rows on unaligned X rows too: parity, Pubmed A/B, host-overhead breakdown of the small shapes
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "hub or narrow or pubmed or golden or timing" > $O/pytest_s28.log 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest_s28.log; exit 1; }
tail -1 $O/pytest_s28.log
timeout -k 10 300 python scripts/ab_tune.py --knob hub_fuse --values 0,1 --shape pubmed --widths F --rounds 30 > $O/hubfuse_pubmed3.log 2>&1 || { tail $O/hubfuse_pubmed3.log; exit 1; }
grep '^{' $O/hubfuse_pubmed3.log
timeout -k 10 300 python scripts/host_overhead.py --shapes cora,pubmed > $O/hostov.log 2>&1 || { tail $O/hostov.log; exit 1; }
grep '^{' $O/hostov.log
