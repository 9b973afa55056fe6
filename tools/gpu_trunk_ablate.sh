set -o pipefail
cd $GRAFT_REPO_ROOT
for opt in "" "--option trunk_dbg=1" "--option trunk_tile=128" "--option trunk_tile=128 --option trunk_dbg=1"; do
echo "== $opt"
timeout -k 10 120 python tools/trunk_bench.py --rays 4096 --samples 128 --iters 5 $opt 2>&1 | grep -v amdgpu.ids
done
