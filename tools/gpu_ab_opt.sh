# Bench line under library options: bash tools/gpu_ab_opt.sh "zsave=0" "zsave=1" ...
# (CONFIG=c5 for the inference line; default the C4 training line; a "lib=libspnerf_amd_x.so"
# token runs that in-tree variant build, sp-nerf_amd/Makefile target variant; EXTRA="--global-batch 512"
# adds bench arguments)
cd $GRAFT_REPO_ROOT
CONFIG=${CONFIG:-c4}
for o in "$@"; do
args=""; lib=libspnerf_amd.so; for kv in $o; do case $kv in lib=*) lib=${kv#lib=};; *) args="$args --option $kv";; esac; done
r=$(SPNERF_AMD_LIB=$lib timeout -k 10 200 python bench.py --config $CONFIG --steps 20 --warmup 5 --no-cpu-baseline --no-secondary $EXTRA $args 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels', {}); print(round(d['ms_per_step'],3), round(d['value']/1e6,2), {c: round(v['ms_per_step'],2) for c, v in k.items() if v['ms_per_step'] > 0.2}, 'frac', round(d['roofline']['frac'],3), 'mlp', round((d.get('mlp_mfma_utilisation') or {}).get('frac', 0),3))")
echo "$CONFIG [$o] ms,Msps=$r"
done
