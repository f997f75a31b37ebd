# GPU: the fuse division without v_div_fmas (common.hpp div_rn): the exhaustive-sample division check,
# bit-identity of whole steps against the previous build (tools/step_hash.py), alternating C2 A/B and
# the per-shape profile of the new build
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-divrn}
timeout -k 10 120 ./tools/div_check > gpurun_out/${tag}_divcheck.txt 2>&1 || { cat gpurun_out/${tag}_divcheck.txt; exit 3; }
cat gpurun_out/${tag}_divcheck.txt
PHX_LIB=libphx_prev.so timeout -k 10 300 python tools/step_hash.py > gpurun_out/${tag}_hash_prev.txt 2>&1 || exit 3
timeout -k 10 300 python tools/step_hash.py > gpurun_out/${tag}_hash_new.txt 2>&1 || exit 3
grep -v amdgpu.ids gpurun_out/${tag}_hash_prev.txt; grep -v amdgpu.ids gpurun_out/${tag}_hash_new.txt
for r in 1 2 3; do
  for L in libphx_prev.so libphx.so; do
    PHX_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-profile > gpurun_out/${tag}_$L.json 2>gpurun_out/${tag}_$L.err || exit 3
    echo "round $r $L: $(python -c "import json;d=json.load(open('gpurun_out/${tag}_$L.json'));print(d['ms_per_step'])")"
  done
done
timeout -k 10 300 python tools/shape_prof.py --top 120 > gpurun_out/${tag}_shapes_c2.txt 2>&1 || exit 3
grep -E "sep_fwd|dw_fwd (32|16|8|4)x|fuse|bwd_other 16x(32|16)" gpurun_out/${tag}_shapes_c2.txt | head -20
