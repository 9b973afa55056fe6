# C4 default line under library options: bash tools/gpu_ab_opt.sh "zsave=0" "zsave=1" ...
cd $GRAFT_REPO_ROOT
for o in "$@"; do
args=""; for kv in $o; do args="$args --option $kv"; done
r=$(timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary $args 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(round(d['ms_per_step'],3), round(d['value']/1e6,2), 'trunk', round(k['trunk_bf16']['ms_per_step'],2), 'nt', round(k['gemm_nt_bf16']['ms_per_step'],2), 'tn', round(k['gemm_tn_bf16']['ms_per_step'],2), 'frac', round(d['roofline']['frac'],3))")
echo "c4 [$o] ms,Msps=$r"
done
