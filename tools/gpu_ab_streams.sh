cd $GRAFT_REPO_ROOT
for mode in "" "--eager"; do for bs in 1 2; do
r=$(timeout -k 10 200 python bench.py --config c4 --global-batch 512 --no-cpu-baseline --no-secondary $mode --option bwd_streams=$bs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3))")
echo "512 mode=[$mode] bwd_streams=$bs ms=$r"
done; done
for bs in 1 2; do
r=$(timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --no-secondary --option bwd_streams=$bs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3))")
echo "4096 graph bwd_streams=$bs ms=$r"
done
