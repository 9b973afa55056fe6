cd $GRAFT_REPO_ROOT
for o in "fused_bwd=0" "fused_bwd=1"; do
r=$(timeout -k 10 200 python bench.py --config c4 --global-batch 512 --steps 30 --warmup 5 --no-cpu-baseline --no-secondary --option $o 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels', {}); print(round(d['ms_per_step'],3), {c: (round(v['ms_per_step'],3), v['launches']) for c, v in k.items()})")
echo "c4@512 [$o] $r"
done
