set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# (1) streaming classifier v2: parity + timings; (2) fused serial hub rows: parity + Pubmed A/B
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "linear or xent or autograd or fused or sgc_model or hub or narrow or pubmed or golden" > $O/pytest_s20.log 2>&1 || { echo PYTEST FAIL; tail -40 $O/pytest_s20.log; exit 1; }
tail -1 $O/pytest_s20.log
for lk in 2 1 2 1; do
  timeout -k 10 200 python -m sgc_amd.classifier_bench --tune linear_kernel=$lk > $O/cls2_lk$lk.log 2>&1 || { tail $O/cls2_lk$lk.log; exit 1; }
  grep -v amdgpu $O/cls2_lk$lk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lk=$lk', 'fwd', round(d['forward']['ms'],4), 'bwd', round(d['backward']['ms'],4), 'closure', round(d['closure']['dropin_ms'],4), 'lbfgs', round(d['lbfgs']['dropin_ms'],2))"
done
timeout -k 10 300 python scripts/ab_tune.py --knob hub_fuse --values 0,1 --shape pubmed --widths F,500 --rounds 20 > $O/hubfuse_pubmed.log 2>&1 || { tail $O/hubfuse_pubmed.log; exit 1; }
grep '^{' $O/hubfuse_pubmed.log
