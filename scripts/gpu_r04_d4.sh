# GPU: C2 A/B after the depthwise revert (3 default bench lines), then the C4 shape profile
# (D4 bf16 1024^2 x 4) and its bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --no-secondary --steps 100 > gpurun_out/ab.json 2> gpurun_out/ab.err
  rc=$?; echo "c2 rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
  [ $rc -eq 0 ] || exit $rc
done
PHX_PROF_DETAIL=1 timeout -k 10 300 python tools/shape_prof.py --model efficientdet-d4 --batch 4 --image-size 1024 --dtype bf16 --top 70 > gpurun_out/shapes_d4_r04.txt 2>&1
rc=$?; echo "shapes rc=$rc"; head -40 gpurun_out/shapes_d4_r04.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model efficientdet-d4 --dtype bf16 --image-size 1024 --batch 4 --steps 50 \
  --no-cpu-baseline --no-secondary > gpurun_out/bench_d4bf16_r04.json 2> gpurun_out/bench_d4bf16_r04.err
rc=$?; echo "d4 rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/bench_d4bf16_r04.json'));print(d['ms_per_step'],d['value'],d['roofline'])"
