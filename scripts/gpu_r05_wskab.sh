# GPU: wave-split-K A/B (PHX_GEMM_WSK 0 / 1) on C2 (3 rounds) and C5 (2 rounds), then the C2 shape profile
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_ab_env3.sh PHX_GEMM_WSK || exit $?
for r in 1 2; do
  for x in 0 1; do
    PHX_GEMM_WSK=$x timeout -k 10 300 python tools/defender_bench.py --no-cpu-baseline --no-profile > gpurun_out/wskd_$x.json 2>/dev/null || exit 1
    echo "C5 round $r PHX_GEMM_WSK=$x: $(python -c "import json;d=json.load(open('gpurun_out/wskd_$x.json'));print(d['ms_per_step'], d['value'])")"
  done
done
timeout -k 10 300 python tools/shape_prof.py --top 80 > gpurun_out/shapes_c2_wsk.txt 2>&1 || { tail -5 gpurun_out/shapes_c2_wsk.txt; exit 1; }
head -40 gpurun_out/shapes_c2_wsk.txt
