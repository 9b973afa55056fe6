# Bench lines under bench.py argument sets, alternating, in one call:
#   bash tools/ab_args.sh "" "--no-reuse-pass1" ...   (REPS rounds, default 2; CONFIG, EXTRA as in gpu_ab_opt.sh)
cd $GRAFT_REPO_ROOT
CONFIG=${CONFIG:-c4}
for r in $(seq ${REPS:-2}); do
for o in "$@"; do
res=$(timeout -k 10 200 python bench.py --config $CONFIG --steps 20 --warmup 5 --no-cpu-baseline --no-secondary $EXTRA $o 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); k=d.get('kernels', {}); print(round(d['ms_per_step'],3), round(d['value']/1e6,2), {c: round(v['ms_per_step'],2) for c, v in k.items() if v['ms_per_step'] > 0.2}, 'frac', round(d['roofline']['frac'],3), 'mlp', round((d.get('mlp_mfma_utilisation') or {}).get('frac', 0),3))") || exit 1
echo "$CONFIG $EXTRA [$o] ms,Msps=$res"
done
done
