# GPU: round-2 evidence of the current step: per-shape launch groups (D0 f32, D4 bf16), a rocprofv3
# kernel-trace summary of the default bench, the D4 bf16 bench line with its roofline
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/shape_prof.py --top 80 > gpurun_out/shapes_d0.txt 2>&1; echo "d0 shapes rc=$?"
timeout -k 10 300 python tools/shape_prof.py --model efficientdet-d4 --batch 4 --dtype bf16 --top 60 > gpurun_out/shapes_d4.txt 2>&1; echo "d4 shapes rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_d0 -o run --output-format csv -- \
  python bench.py --no-cpu-baseline --steps 5 --warmup 2 --no-profile > gpurun_out/prof_d0.log 2>&1
rc=$?; echo "rocprof d0 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16 --no-cpu-baseline \
  > gpurun_out/bench_d4.json 2> gpurun_out/bench_d4.err
rc=$?; echo "bench d4 rc=$rc"; cat gpurun_out/bench_d4.json
