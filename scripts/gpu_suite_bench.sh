# GPU: the whole -m gpu suite, bench lines (D0 C2, D4 C4 bf16 and fp32), rocprof kernel traces
# (rocpd databases; summarise with tools/rocpd_stats.py) and the per-shape launch-group tables
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/pytest.log | tail -8
[ $rc -le 1 ] || exit $rc
for args in "" "--model efficientdet-d4 --image-size 1024 --batch 4 --steps 10 --warmup 2 --dtype bf16" "--model efficientdet-d4 --image-size 1024 --batch 4 --steps 10 --warmup 2"; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile $args > gpurun_out/ab.json 2> gpurun_out/ab.err
  rc=$?; echo "[$args] rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_d0 -o run -- python bench.py --no-cpu-baseline --no-profile --steps 10 --warmup 2 > /dev/null 2>&1
rc=$?; echo "prof d0 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_d4 -o run -- python bench.py --no-cpu-baseline --no-profile --model efficientdet-d4 --image-size 1024 --batch 4 --steps 5 --warmup 1 --dtype bf16 > /dev/null 2>&1
rc=$?; echo "prof d4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/shape_prof.py --top 80 > gpurun_out/shapes_d0.txt 2>&1; echo "shapes d0 rc=$?"
