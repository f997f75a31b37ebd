# GPU: kernel trace of the reference's placement flow (first-pass boxes, person prior 4.6, the next
# batch's first pass beside each step): per-kernel totals and the launch timeline of one step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-fp}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/ktfp -o run --output-format csv -- python bench.py --steps 10 --warmup 2 \
  --placement first-pass --person-bias 4.6 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_kt.log || exit 3
python -c "import json;d=json.load(open('gpurun_out/${tag}_bench.json'));print('first-pass flow', d['ms_per_step'], d['value'])"
f=$(find /tmp/ktfp -name '*kernel_trace.csv' | head -1); s=$(find /tmp/ktfp -name '*kernel_stats.csv' | head -1)
cp "$s" gpurun_out/${tag}_kernel_stats.csv
python tools/kt_summary.py "$f" eot > gpurun_out/${tag}_eot.txt
python tools/kt_summary.py "$f" > gpurun_out/${tag}_kt_summary.txt
head -30 gpurun_out/${tag}_eot.txt
