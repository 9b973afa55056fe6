# round 3 (session 3): packed sine epilogue in the DMA NT GEMM — bitwise tests vs the SPN_PK_EPI 0 build, A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_variants.py tests/test_gpu_trunk.py -x -v --timeout 200 --timeout-method thread -k "epilogue or layerwise or register_d" > gpurun_out/r3r_tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error|assert" gpurun_out/r3r_tests.log | head -20; tail -5 gpurun_out/r3r_tests.log; exit 1; }
tail -1 gpurun_out/r3r_tests.log
# bitwise: one training render + gradients under both builds
for lib in libspnerf_amd.so libspnerf_amd_nopk.so; do
SPNERF_AMD_LIB=$lib timeout -k 10 200 python3 - <<'PY' || exit 1
import os, sys, torch
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from test_gpu_variants import _render_bf16
r, g = _render_bf16({}, n=300)
torch.save({"r": r, "g": g}, f"gpurun_out/r3r_{os.environ['SPNERF_AMD_LIB']}.pt")
PY
done
python3 - <<'PY'
import torch
a = torch.load("gpurun_out/r3r_libspnerf_amd.so.pt"); b = torch.load("gpurun_out/r3r_libspnerf_amd_nopk.so.pt")
bad = [k for k in a["r"] if not torch.equal(a["r"][k], b["r"][k])] + [k for k in a["g"] if not torch.equal(a["g"][k], b["g"][k])]
print("packed vs scalar epilogue build: bitwise", not bad, bad[:5])
PY
bash tools/gpu_ab_opt.sh "lib=libspnerf_amd_nopk.so" "trunk2=3" "lib=libspnerf_amd_nopk.so" "trunk2=3"
