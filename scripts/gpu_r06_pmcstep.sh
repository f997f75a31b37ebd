# GPU: HBM traffic of a whole C2 step from PMC counters (FETCH_SIZE / WRITE_SIZE in separate passes,
# every kernel), with the fused separable convs (PHX_SEP=1, default) and without (PHX_SEP=0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
CMD="python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-secondary"
for x in 1 0; do
  for c in FETCH_SIZE WRITE_SIZE; do
    PHX_SEP=$x timeout -k 10 300 rocprofv3 --pmc $c -d gpurun_out/pmcstep_${x}_$c -o run --output-format csv -- $CMD \
      > gpurun_out/pmcstep_${x}_$c.log 2>&1 || exit 3
  done
  echo "PHX_SEP=$x: $(python tools/pmc_step.py gpurun_out/pmcstep_${x}_FETCH_SIZE gpurun_out/pmcstep_${x}_WRITE_SIZE 3 | head -3)"
done
