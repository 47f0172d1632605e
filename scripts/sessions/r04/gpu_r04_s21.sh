set -o pipefail
O=gpurun_out/r04; mkdir -p $O
# streaming classifier v2 diagnostics + counters; Pubmed hop kernel trace with and without the fused hub rows
for lk in 3 4 2; do
  timeout -k 10 200 python -m sgc_amd.classifier_bench --tune linear_kernel=$lk > $O/cls3_diag_lk$lk.log 2>&1 || { tail $O/cls3_diag_lk$lk.log; exit 1; }
  grep -v amdgpu $O/cls3_diag_lk$lk.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lk=$lk', 'fwd', round(d['forward']['ms'],4))"
done
bash scripts/pmc_classifier.sh > $O/pmc_cls6.log 2>&1 || { cat $O/pmc_cls6.log; exit 1; }
cat gpurun_out/pmc_cls/sq.summary gpurun_out/pmc_cls/insts.summary gpurun_out/pmc_cls/lds.summary | grep -E 'linear_stream'
cd /tmp && export TMPDIR=/tmp
for f in 0 1; do
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_pubmed_fuse$f -o p -- python3 $GRAFT_REPO_ROOT/scripts/ab_tune.py --knob hub_fuse --values $f,$f --shape pubmed --widths 500 --rounds 10 > $GRAFT_REPO_ROOT/$O/prof_pubmed_fuse$f.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/prof_pubmed_fuse$f.log; exit 1; }
find $GRAFT_REPO_ROOT/$O/prof_pubmed_fuse$f -name "*kernel_stats.csv" -exec cut -c1-200 {} \; | head -8
done
