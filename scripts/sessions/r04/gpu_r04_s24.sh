set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# classifier v4 (batched W staging) + fused serial hub rows in the csr kernel: parity, timings, Pubmed A/B
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "linear or xent or autograd or fused or sgc_model or hub or narrow or pubmed or golden" > $O/pytest_s24.log 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest_s24.log; exit 1; }
tail -1 $O/pytest_s24.log
for lk in 2 4 3 1 2 4 3 1; do
  timeout -k 10 200 python -m sgc_amd.classifier_bench --tune linear_kernel=$lk > $O/cls5_lk$lk.log 2>&1 || { tail $O/cls5_lk$lk.log; exit 1; }
  grep -v amdgpu $O/cls5_lk$lk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lk=$lk', 'fwd', round(d['forward']['ms'],4))"
done
timeout -k 10 300 python scripts/ab_tune.py --knob hub_fuse --values 0,1 --shape pubmed --widths F,500 --rounds 20 > $O/hubfuse_pubmed2.log 2>&1 || { tail $O/hubfuse_pubmed2.log; exit 1; }
grep '^{' $O/hubfuse_pubmed2.log
