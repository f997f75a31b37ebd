# GPU: the fold test, the C4 line with / without the in-launch finalize, a kernel trace of the first-pass flow
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fin.py -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/fin3.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/fin3.log; grep -E "FAILED|Error|^E " gpurun_out/fin3.log | head -20
[ $rc -eq 0 ] || exit $rc
D4="--model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16"
for r in 1 2; do
for x in 8192 0; do
  PHX_FIN_MAX=$x timeout -k 10 300 python bench.py $D4 --steps 60 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/c4fin_$x.json 2>/dev/null || exit 1
  echo "C4 PHX_FIN_MAX=$x: $(python -c "import json;d=json.load(open('gpurun_out/c4fin_$x.json'));print(d['ms_per_step'], d['value'])")"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/secprof -o run --output-format csv -- python3 bench.py --placement first-pass --person-bias 4.6 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/secprof.log 2>&1 || { tail -20 gpurun_out/secprof.log; exit 1; }
grep -h '"metric"' gpurun_out/secprof.log | cut -c1-200
