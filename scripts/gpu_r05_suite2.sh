# GPU: the whole -m gpu suite, then the C4 line with and without the in-launch finalize
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1500 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/suite2.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/suite2.log; grep -E "FAILED|Error" gpurun_out/suite2.log | head -20
[ $rc -eq 0 ] || exit $rc
D4="--model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16"
for x in 8192 0; do
  PHX_FIN_MAX=$x timeout -k 10 300 python bench.py $D4 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/c4fin_$x.json 2>/dev/null || exit 1
  echo "C4 PHX_FIN_MAX=$x: $(python -c "import json;d=json.load(open('gpurun_out/c4fin_$x.json'));print(d['ms_per_step'], d['value'])")"
done
