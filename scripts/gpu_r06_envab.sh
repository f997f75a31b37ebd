# GPU: environment knob A/B on the current build — per-shape groups of one step for the base and each
# variant (tools/shape_prof.py), then alternating C2 bench rounds.  $2... = the variants, each one
# assignment (e.g. PHX_DW_S2RPT=1) or several joined by commas (PHX_A=1,PHX_B=2).  SHAPE_ARGS / BENCH_ARGS
# select another configuration (e.g. the C4 line's --model efficientdet-d4 --batch 4 ...)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-envab}
shift
vars=("BASE=1" "$@")
i=0
for v in "${vars[@]}"; do
  timeout -k 10 200 env ${v//,/ } python tools/shape_prof.py --top 60 $SHAPE_ARGS > gpurun_out/${tag}_shapes_$i.txt 2>&1 || exit 3
  i=$((i+1))
done
for r in 1 2 3; do
  line="round $r:"
  i=0
  for v in "${vars[@]}"; do
    timeout -k 10 200 env ${v//,/ } python bench.py $BENCH_ARGS --no-cpu-baseline --no-secondary --no-profile > gpurun_out/${tag}_$i.json 2>gpurun_out/${tag}_$i.err || exit 3
    line="$line  $v $(python -c "import json;print(json.load(open('gpurun_out/${tag}_$i.json'))['ms_per_step'])")"
    i=$((i+1))
  done
  echo "$line"
done
