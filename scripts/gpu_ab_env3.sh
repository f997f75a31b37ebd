# GPU: A/B of an environment switch on the default bench (alternating, 3 rounds).
# usage: bash scripts/gpu_ab_env3.sh VAR [bench args...]   (runs VAR=0 and VAR=1)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
VAR=$1
shift
for r in 1 2 3; do
  for v in 0 1; do
    env "$VAR=$v" timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --no-secondary --steps 100 "$@" \
      > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?; echo "$VAR=$v rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
