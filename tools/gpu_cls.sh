# per-class kernel times (ms per step) of the C4 line under several libraries: CLS="a b" names the
# classes shown; EXTRA adds bench arguments
cd $GRAFT_REPO_ROOT
for lib in "$@"; do
r=$(SPNERF_AMD_LIB=$lib timeout -k 10 200 python bench.py --config c4 --steps 20 --warmup 5 --no-cpu-baseline --no-secondary $EXTRA 2>/dev/null | CLS="$CLS" python -c "
import json, os, sys
d = json.loads(sys.stdin.read()); k = d.get('kernels', {}); want = os.environ['CLS'].split()
print(round(d['ms_per_step'], 3), {c: round(v['ms_per_step'], 4) for c, v in k.items() if c in want})")
echo "$lib $EXTRA $r"
done
