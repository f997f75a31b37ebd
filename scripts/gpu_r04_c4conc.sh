# GPU: C4 (D4 bf16 1024^2 x4) step time — concurrent first pass at the default fork point, at half
# the ops (PHX_FORK_FRAC=0.5), and off (PHX_CONC=0).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for e in PHX_X=1 PHX_FORK_FRAC=0.5 PHX_CONC=0; do
  env $e timeout -k 10 300 python bench.py --model efficientdet-d4 --dtype bf16 --image-size 1024 --batch 4 --steps 30 \
    --no-cpu-baseline --no-profile --no-secondary > gpurun_out/c4c.json 2> gpurun_out/c4c.err
  echo "$e rc=$? $(python -c "import json;d=json.load(open('gpurun_out/c4c.json'));print(d['ms_per_step'],d['value'])")"
done
