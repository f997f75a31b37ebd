# GPU: sweep of environment tuning knobs on the default bench (each config vs the default, 2 rounds).
# usage: bash scripts/gpu_sweep_env.sh "VAR=a" "VAR=b VAR2=c" ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "BASE=1" "$@"; do
    env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --no-secondary --steps 100 \
      > gpurun_out/sw.json 2> gpurun_out/sw.err
    rc=$?; echo "[$cfg] rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/sw.json'));print(d['ms_per_step'],d['value'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
