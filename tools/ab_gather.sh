cd $GRAFT_REPO_ROOT
for f in "" "--torch-gather" "" "--torch-gather"; do
r=$(timeout -k 10 200 python bench.py --config c4 --global-batch 512 --steps 30 --warmup 5 --no-cpu-baseline --no-secondary $f 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3))")
echo "c4@512 [$f] $r"
done
