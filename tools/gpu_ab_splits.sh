cd $GRAFT_REPO_ROOT
for gb in 512 4096; do for mp in 1024 2048 4096; do
r=$(timeout -k 10 200 python bench.py --config c4 --global-batch $gb --no-cpu-baseline --no-secondary --option tn_bf16_min_points=$mp 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3))")
echo "gb=$gb min_points=$mp ms=$r"
done; done
