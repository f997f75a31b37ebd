# GPU: A/B of an alternative in-tree build (PHX_LIB) on the default bench, alternating, 3 rounds;
# then the per-shape launch groups of both builds (PHX_AB_SHAPES=1).
# usage: bash scripts/gpu_ab_lib.sh libphx_x.so
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for lib in libphx.so "$1"; do
    PHX_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --no-secondary --steps 100 \
      > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?; echo "$lib rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
[ -n "${PHX_AB_SHAPES:-}" ] || exit 0
for lib in libphx.so "$1"; do
  PHX_LIB=$lib timeout -k 10 300 python tools/shape_prof.py --top 40 > gpurun_out/shapes_$lib.txt 2>&1 || exit $?
done
