# Weight-gradient lab + bench pairs under TN options: bash tools/ab_tn.sh "tn_bf16_m16=0" "tn_bf16_m16=1" ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
make -C tools tn_lab > gpurun_out/tn_lab_build.log 2>&1 || { tail -5 gpurun_out/tn_lab_build.log; exit 1; }
timeout -k 10 120 ./tools/tn_lab 1048576 20 || exit 1
bash tools/gpu_ab_opt.sh "$@"
