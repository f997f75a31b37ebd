# GPU: C2 fork point of the concurrent first pass — default (stage 6) against PHX_FORK_FRAC fractions
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for f in def 0.2 0.3 0.45 0.6; do
    if [ $f = def ]; then unset PHX_FORK_FRAC; else export PHX_FORK_FRAC=$f; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --no-secondary --steps 100 > gpurun_out/ff.json 2>/dev/null || exit 1
    echo "round $r fork $f: $(python -c "import json;d=json.load(open('gpurun_out/ff.json'));print(d['ms_per_step'])")"
  done
done
