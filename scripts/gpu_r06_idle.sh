# GPU: idle time of the concurrent C2 step (the default bench configuration) from a kernel trace over
# all streams (tools/idle_gaps.py): the last 10 steps' window
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-idle}
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/idl -o run --output-format csv -- python bench.py --steps 20 --warmup 3 \
  --no-cpu-baseline --no-secondary --no-profile > gpurun_out/${tag}_bench.log 2>&1 || exit 3
f=$(find /tmp/idl -name '*kernel_trace.csv' | head -1)
python tools/idle_gaps.py "$f" --last 100000 --top 30 > gpurun_out/${tag}_gaps.txt
cat gpurun_out/${tag}_gaps.txt | head -34
