# round-3 batch 2: C5 with the two-workgroup trunk for inference (trunk2=3) and the full
# long-horizon PSNR study
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CONFIG=c5 bash tools/gpu_ab_opt.sh "trunk2=0" "trunk2=3" "trunk2=0" "trunk2=3" > gpurun_out/r3d_c5_trunk2.log 2>&1
timeout -k 10 700 python -u -c "
import json, bench
r = bench.psnr_long()
print(json.dumps(r))
" > gpurun_out/r3d_psnr_long.json 2> gpurun_out/r3d_psnr_long.err
