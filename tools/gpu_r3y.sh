# round 3 (session 3): bench step gathering each per-ray field once (bench.py) vs the previous step (bench_prev.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
for b in bench_prev.py bench.py bench_prev.py bench.py; do
r=$(timeout -k 10 200 python $b --config c4 --global-batch 512 --steps 30 --warmup 5 --no-cpu-baseline --no-secondary 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3))") || exit 1
echo "c4@512 $b $r"
done
for b in bench_prev.py bench.py; do
r=$(timeout -k 10 200 python $b --config c4 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3))") || exit 1
echo "c4 $b $r"
done
timeout -k 10 300 python bench.py --gpus 2 --share-device --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > gpurun_out/r3y_dp2.json 2> gpurun_out/r3y_dp2.err || { tail -20 gpurun_out/r3y_dp2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r3y_dp2.json')); print('dp2 share-device', d['ms_per_step'], d['value'], d.get('allreduce_ms_per_step'))"
