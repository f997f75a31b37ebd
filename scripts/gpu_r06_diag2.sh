# GPU: the bf16 wave-split-K layer diagnosis (scripts/diag_bf16_wsk_layers.py), per-shape profiles of
# C2 and C4 on the current build, and a kernel trace of C2 for the launch count per step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-d2}
timeout -k 10 900 python -u scripts/diag_bf16_wsk_layers.py > gpurun_out/${tag}_bf16wsk.txt 2>&1 || exit 3
tail -8 gpurun_out/${tag}_bf16wsk.txt
timeout -k 10 300 python tools/shape_prof.py --top 120 > gpurun_out/${tag}_shapes_c2.txt 2>&1 || exit 3
timeout -k 10 300 python tools/shape_prof.py --model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16 --top 80 \
  > gpurun_out/${tag}_shapes_d4bf16.txt 2>&1 || exit 3
PHX_CONC=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt -o run --output-format csv -- python bench.py --steps 10 --warmup 2 \
  --no-cpu-baseline --no-secondary --no-profile > gpurun_out/${tag}_kt.log 2>&1 || exit 3
f=$(find /tmp/kt -name '*kernel_trace.csv' | head -1); s=$(find /tmp/kt -name '*kernel_stats.csv' | head -1)
cp "$s" gpurun_out/${tag}_kernel_stats_c2.csv
python tools/kt_summary.py "$f" > gpurun_out/${tag}_kt_summary.txt
echo "kernel launches in trace: $(($(wc -l < "$f") - 1)) (12 steps + setup)"
