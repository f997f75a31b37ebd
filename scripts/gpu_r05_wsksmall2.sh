# GPU: C2 A/B of PHX_GEMM_WSK_SMALL 0 / 1 (alternating, three rounds)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for x in 0 1; do
    PHX_GEMM_WSK_SMALL=$x timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --no-secondary --steps 100 > gpurun_out/wsm_$x.json 2>/dev/null || exit 1
    echo "C2 round $r WSK_SMALL=$x: $(python -c "import json;d=json.load(open('gpurun_out/wsm_$x.json'));print(d['ms_per_step'])")"
  done
done
