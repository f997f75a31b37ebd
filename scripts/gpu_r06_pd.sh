# GPU (round 6): the 16-wide GEMM's prefetch depth (PHX_GEMM_PD builds libphx_pd{2,3,4,6}.so against
# libphx.so): bit-identity of the step (tools/step_hash.py), the N = 16 launch groups
# (tools/shape_prof.py), then an alternating C2 bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for L in libphx.so libphx_pd2.so libphx_pd3.so libphx_pd4.so libphx_pd6.so; do
  PHX_LIB=$L timeout -k 10 200 python tools/step_hash.py > gpurun_out/pd_hash_$L.txt 2>&1 || { tail -5 gpurun_out/pd_hash_$L.txt; exit 3; }
  echo "$L hash: $(tr '\n' ' ' < gpurun_out/pd_hash_$L.txt)"
  PHX_LIB=$L timeout -k 10 200 python tools/shape_prof.py --top 200 > gpurun_out/pd_shapes_$L.txt 2>&1 || { tail -5 gpurun_out/pd_shapes_$L.txt; exit 3; }
  grep -E "N=16 " gpurun_out/pd_shapes_$L.txt || true
done
for r in 1 2; do
  for L in libphx.so libphx_pd2.so libphx_pd3.so libphx_pd4.so libphx_pd6.so; do
    PHX_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-profile > gpurun_out/pd_ab_$L.json 2>gpurun_out/pd_ab_$L.err || exit 3
    echo "round $r $L: $(python -c "import json;d=json.load(open('gpurun_out/pd_ab_$L.json'));print(d['ms_per_step'])")"
  done
done
