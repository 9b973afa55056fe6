# Socket power, shader clock and junction temperature sampled by rocm-smi (≈0.6 s per sample) while
# bench.py runs a long line; per workload into gpurun_out/pw/<name>.txt.
#     bash tools/power_probe.sh            (C4 400 steps, C5 200 steps)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pw
probe() {  # name, bench args
  local name=$1; shift
  (timeout -k 10 300 python bench.py "$@" --no-cpu-baseline --no-secondary > gpurun_out/pw/$name.json 2> gpurun_out/pw/$name.err) &
  local bp=$!
  for i in $(seq 1 400); do
    (date +%s.%N; rocm-smi --showpower --showclocks --showtemp 2>&1 | grep -E "Package Power|sclk|junction") >> gpurun_out/pw/$name.txt
    kill -0 $bp 2>/dev/null || break
  done
  wait $bp || return 1
}
probe c4 --steps 400 --warmup 5 && probe c5 --config c5 --steps 200 --warmup 3
