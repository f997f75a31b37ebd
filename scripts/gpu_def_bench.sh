# GPU: defender (C5) bench lines at 8 and 24 images/GPU, then a rocprofv3 kernel-trace summary of the 8-image run
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/defender_bench.py --batch 8 > gpurun_out/def_b8.json 2> gpurun_out/def_b8.err
rc=$?; echo "def b8 rc=$rc"; cat gpurun_out/def_b8.json; tail -3 gpurun_out/def_b8.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/defender_bench.py --batch 24 > gpurun_out/def_b24.json 2> gpurun_out/def_b24.err
rc=$?; echo "def b24 rc=$rc"; cat gpurun_out/def_b24.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_def -o run --output-format csv -- \
  python tools/defender_bench.py --batch 8 --steps 5 > gpurun_out/prof_def.log 2>&1
echo "rocprof def rc=$?"
