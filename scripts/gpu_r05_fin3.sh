# GPU: in-launch BN finalize on the wave-split-K build — its parity test, then C2 / C4 A/B of
# PHX_FIN_MAX 0 / 8192 (alternating, two rounds)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_fin.py > gpurun_out/fin3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/fin3_tests.log; grep -E "FAILED|^E " gpurun_out/fin3_tests.log | head; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for x in 0 8192; do
    PHX_FIN_MAX=$x timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --no-secondary --steps 100 > gpurun_out/fin3_$x.json 2>/dev/null || exit 1
    echo "C2 round $r PHX_FIN_MAX=$x: $(python -c "import json;d=json.load(open('gpurun_out/fin3_$x.json'));print(d['ms_per_step'])")"
  done
done
for x in 0 8192; do
  PHX_FIN_MAX=$x timeout -k 10 300 python bench.py --model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16 --steps 30 \
    --no-cpu-baseline --no-profile --no-secondary > gpurun_out/fin3d4_$x.json 2>/dev/null || exit 1
  echo "C4 PHX_FIN_MAX=$x: $(python -c "import json;d=json.load(open('gpurun_out/fin3d4_$x.json'));print(d['ms_per_step'])")"
done
