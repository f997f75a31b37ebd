# GPU: D4 1024x1024 bench line (no tests, no CPU leg) under several environment settings
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for setting in "$@"; do
  env $setting timeout -k 10 300 python bench.py --model efficientdet-d4 --image-size 1024 --batch 4 --steps 5 \
    --warmup 2 --no-cpu-baseline --no-profile > gpurun_out/bench_ab.json 2> gpurun_out/bench_ab.err
  rc=$?; echo "[$setting] rc=$rc $(python -c 'import json;d=json.load(open("gpurun_out/bench_ab.json"));print(d["value"],d["ms_per_step"])')"
  [ $rc -eq 0 ] || exit $rc
done
