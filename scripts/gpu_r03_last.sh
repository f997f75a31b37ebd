# GPU: the last round-3 checks — the defender with and without the opt-in weight-gradient side
# stream (tests + bench A/B), the forward-only-executor variant (PHX_LIB=libphx_slim.so: concurrency
# tests, full-size parity, workspace), then the whole -m gpu suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
PHX_DEF_CONC=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_defender.py \
  tests/test_gpu_defender_512.py tests/test_gpu_defender_distributed.py > gpurun_out/pytest_def.log 2>&1
echo "def conc tests rc=$?"
for e in PHX_DEF_CONC=0 PHX_DEF_CONC=1 PHX_DEF_CONC=0 PHX_DEF_CONC=1; do
  env $e timeout -k 10 300 python tools/defender_bench.py > gpurun_out/def.json 2>/dev/null
  echo "$e def rc=$? $(python -c "import json;d=json.load(open('gpurun_out/def.json'));print(d['ms_per_step'], d['value'])")"
done
PHX_LIB=libphx_slim.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_concurrent.py tests/test_gpu_fullsize.py > gpurun_out/pytest_slim.log 2>&1
echo "slim tests rc=$?"
PHX_LIB=libphx_slim.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary > gpurun_out/b_slim.json 2>/dev/null
echo "slim bench rc=$? $(python -c "import json;d=json.load(open('gpurun_out/b_slim.json'));print(d['ms_per_step'], d['config']['workspace_gb_per_gpu'])")"
PHX_NO_BENCH=1 bash scripts/gpu_r03_tests.sh
