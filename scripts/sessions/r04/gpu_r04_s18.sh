set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# streaming forward diagnostics: full / loads only / MFMA only / LDS tile, forward ms each
for lk in 2 3 4 1 2 3 4 1; do
  timeout -k 10 200 python -m sgc_amd.classifier_bench --tune linear_kernel=$lk > $O/cls_diag_lk$lk.log 2>&1 || { tail $O/cls_diag_lk$lk.log; exit 1; }
  grep -v amdgpu $O/cls_diag_lk$lk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lk=$lk', 'fwd', round(d['forward']['ms'],4))"
done
bash scripts/pmc_classifier.sh > $O/pmc_cls4.log 2>&1 || { cat $O/pmc_cls4.log; exit 1; }
cat gpurun_out/pmc_cls/sq.summary gpurun_out/pmc_cls/insts.summary gpurun_out/pmc_cls/lds.summary gpurun_out/pmc_cls/fetch.summary | grep -E 'linear_stream'
