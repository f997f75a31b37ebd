# GPU: EOT v2 kernels — bit-identity vs v1, the EOT / first-pass parity tests, first-pass-flow A/B and kernel times
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_eot_v2.py tests/test_gpu_eot_edges.py tests/test_gpu_firstpass.py tests/test_gpu_defender.py \
  -x -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/eot_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/eot_tests.log; grep -E "FAILED|Error|^E " gpurun_out/eot_tests.log | head -20
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for x in 0 1; do
    PHX_EOT_V1=$x timeout -k 10 300 python bench.py --placement first-pass --person-bias 4.6 --steps 50 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/eot_$x.json 2>/dev/null || exit 1
    echo "round $r PHX_EOT_V1=$x: $(python -c "import json;d=json.load(open('gpurun_out/eot_$x.json'));print(d['ms_per_step'], d['value'], d['config']['patches_per_step'])")"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/eotprof -o run --output-format csv -- python3 bench.py --placement first-pass --person-bias 4.6 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/eotprof.log 2>&1 || { tail -20 gpurun_out/eotprof.log; exit 1; }
grep -h "k_eot" gpurun_out/eotprof/run_kernel_stats.csv | cut -d, -f1-4
