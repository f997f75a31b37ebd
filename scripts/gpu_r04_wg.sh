# GPU: defender weight-gradient variants (row steps in flight U = 4 / 8, row-slice cap 256 / 1024) on
# C5 (tools/defender_bench.py), alternating, then the round-4 final evidence (scripts/gpu_r04_final.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for v in "" _u8 _s1k _u8s1k; do
    PHX_LIB=libphx$v.so timeout -k 10 300 python tools/defender_bench.py --no-cpu-baseline --no-profile --steps 50 > gpurun_out/abd.json 2> gpurun_out/abd.err
    rc=$?; echo "c5 lib$v rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/abd.json'));print(d['ms_per_step'],d['value'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
bash scripts/gpu_r04_final.sh
