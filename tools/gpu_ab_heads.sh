cd $GRAFT_REPO_ROOT
for fh in 1 0; do
r=$(timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline --option fused_heads=$fh 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3), round(d['value']/1e6,1), round(d['mlp_gemms']['frac'],3))")
echo "c5 fused_heads=$fh ms,Msps,mlp_frac=$r"
done
timeout -k 10 200 python tools/trunk_bench.py --rays 4096 --samples 128 --iters 5 2>&1 | grep -v amdgpu
