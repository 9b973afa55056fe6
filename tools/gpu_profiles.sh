# Round profiles: PMC traffic (C4 at 4096 and 512 rays per rank, C3, C5), then rocprofv3 kernel
# stats of the C4 workload alone (no CPU leg, no C2, no PSNR studies: one shape per kernel class),
# of C4 at 512 rays and of C5, each with its per-launch-shape table (tools/trace_shapes.py).
# Traces stay in /tmp; the stats CSVs, shape tables and bench JSON land in gpurun_out/prof
# (copied to profiles/<round>/ by hand).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
bash tools/pmc_bench.sh c4:4096 c4:512 c3:1024 c5:32768 || exit 1
KEYS="k_gemm_tn_bf16d k_trunk_bf16 k_trunk_bwd_bf16 k_gemm_nt_bf16d k_trunk2_bf16 k_heads_bf16 k_reduce_slabs_multi k_gemm_tn_bf16_k64"
prof() {  # name, timeout, bench args
  local name=$1 t=$2; shift 2
  timeout -k 10 $t rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$name -o p -- python3 bench.py "$@" > gpurun_out/prof/$name.json 2> gpurun_out/prof/$name.err || { tail gpurun_out/prof/$name.err; return 1; }
  cp $(find /tmp/prof_$name -name "*kernel_stats.csv" -print -quit) gpurun_out/prof/${name}_kernel_stats.csv &&
  python3 tools/trace_shapes.py $(find /tmp/prof_$name -name "*kernel_trace.csv" -print -quit) $KEYS > gpurun_out/prof/${name}_shapes.txt
}
prof c4 400 --no-cpu-baseline --no-secondary &&
prof c4_512 300 --global-batch 512 --steps 30 --no-cpu-baseline --no-secondary &&
prof c5 300 --config c5 --steps 10 --warmup 3 || exit 1
echo done
