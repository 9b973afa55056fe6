# C4 at a small global batch (default 512 rays: the per-rank work of 8 GPUs) under library
# options, pairs in one call:  GB=512 bash tools/ab512.sh "fused_bwd=0" "fused_bwd=1" ...
# (a "lib=libspnerf_amd_x.so" token runs that in-tree variant build, as tools/gpu_ab_opt.sh)
cd $GRAFT_REPO_ROOT
GB=${GB:-512}
for o in "$@"; do
args=""; lib=libspnerf_amd.so; for kv in $o; do case $kv in lib=*) lib=${kv#lib=};; *) args="$args --option $kv";; esac; done
r=$(SPNERF_AMD_LIB=$lib timeout -k 10 200 python bench.py --config c4 --global-batch $GB --steps 30 --warmup 5 --no-cpu-baseline --no-secondary $args 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels', {}); print(round(d['ms_per_step'],3), {c: (round(v['ms_per_step'],3), v['launches']) for c, v in k.items() if v['ms_per_step'] > 0.05})")
echo "c4@$GB [$o] $r"
done
