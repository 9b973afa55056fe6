# C4 default line with the bf16 NT GEMM variants (option nt_bf16_variant)
cd $GRAFT_REPO_ROOT
for v in "$@"; do
r=$(timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --option nt_bf16_variant=$v 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print(round(d['ms_per_step'],3), round(d['value']/1e6,2), round(k['gemm_nt_bf16']['avg_us'],1), round(k['gemm_nt_bf16']['ms_per_step'],2), round(d['roofline']['frac'],3))")
echo "c4 nt_bf16_variant=$v ms,Msps,nt_avg_us,nt_ms,frac=$r"
done
