set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
CONFIG=c5 bash tools/gpu_ab_opt.sh "" "trunk2_tile=64" "" "trunk2_tile=64" > gpurun_out/r3f_ab.log 2>&1
bash tools/ab512.sh "" "nt_bf16_ip_gen=0" "" "nt_bf16_ip_gen=0" >> gpurun_out/r3f_ab.log 2>&1
GB=4096 bash tools/ab512.sh "" "nt_bf16_ip_gen=0" "" "nt_bf16_ip_gen=0" >> gpurun_out/r3f_ab.log 2>&1
