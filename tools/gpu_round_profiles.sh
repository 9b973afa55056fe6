# Round evidence beyond the suite: the bench lines of C4 at 512 rays, C3 and C5, then
# tools/gpu_profiles.sh (PMC HBM traffic per kernel class + rocprofv3 kernel stats) and the SQ
# counters of the C4 step (tools/pmc_c4.sh).  Usage: bash tools/gpu_round_profiles.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-prof}
mkdir -p gpurun_out/$T
timeout -k 10 200 python bench.py --config c4 --global-batch 512 --no-cpu-baseline --no-secondary > gpurun_out/$T/bench_c4_512.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline --no-secondary > gpurun_out/$T/bench_c3.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline --no-secondary > gpurun_out/$T/bench_c5.json 2>/dev/null || exit 1
for f in c4_512 c3 c5; do python -c "import json; d=json.load(open('gpurun_out/$T/bench_$f.json')); print('$f', round(d['ms_per_step'],3), round(d['value']/1e6,2), d['roofline']['kernel'][:22], round(d['roofline']['frac'],3), (d.get('mlp_mfma_utilisation') or {}).get('frac'))"; done
bash tools/gpu_profiles.sh || exit 1
bash tools/pmc_c4.sh > /dev/null && cp gpurun_out/pmc_c4/summary.txt gpurun_out/$T/pmc_c4_sq.txt || exit 1
GB=512 bash tools/pmc_c4.sh > /dev/null && cp gpurun_out/pmc_c4/summary.txt gpurun_out/$T/pmc_c4_512_sq.txt
echo done
