# save-mode trunk: 64- vs 128-point tiles, with and without the HBM copy-outs (trunk_dbg=1)
cd $GRAFT_REPO_ROOT
for o in "trunk_tile=64" "trunk_tile=128" "trunk_tile=64 --option trunk_dbg=1" "trunk_tile=128 --option trunk_dbg=1"; do
echo "== $o"
timeout -k 10 120 python tools/trunk_bench.py --rays 4096 --samples 128 --iters 5 --option $o 2>&1 | grep -E "^save|^nosave"
done
