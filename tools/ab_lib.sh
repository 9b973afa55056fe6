#!/bin/bash
# Same-call A/B of two builds of the library: the committed tree's libspnerf_amd.so against an
# earlier build saved as sp-nerf_amd/libspnerf_amd_prev.so (git stash; make -C sp-nerf_amd variant
# VDEF= VLIB=libspnerf_amd_prev.so; git stash pop), C4 and C4 at 512 rays, alternating.
#     bash tools/ab_lib.sh [rounds]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for r in $(seq ${1:-2}); do
  for lib in prev cur; do
    if [ $lib = prev ]; then export SPNERF_AMD_LIB=libspnerf_amd_prev.so; else unset SPNERF_AMD_LIB; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/ab/c4_$lib.json 2>/dev/null || exit 1
    timeout -k 10 200 python bench.py --global-batch 512 --no-cpu-baseline --no-secondary > gpurun_out/ab/c4_512_$lib.json 2>/dev/null || exit 1
    python -c "
import json; a=json.load(open('gpurun_out/ab/c4_$lib.json')); b=json.load(open('gpurun_out/ab/c4_512_$lib.json'))
k=a['kernels']; print('$lib', 'c4', round(a['ms_per_step'],3), 'c4@512', round(b['ms_per_step'],3), {n: round(k[n]['ms_per_step'],3) for n in ('trunk_bf16_train','heads_train','trunk_bwd_bf16','gemm_tn_bf16d','gemm_nt_bf16d','gemm_nt_bf16d_dmul') if n in k})"
  done
done
