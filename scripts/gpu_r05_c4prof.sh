# GPU: C4 kernel trace (D4 1024^2 x 4 bf16, well-conditioned draw)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
D4="--model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/c4prof -o run --output-format csv -- python3 bench.py $D4 --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/c4prof.log 2>&1 || { tail -20 gpurun_out/c4prof.log; exit 1; }
grep -h '"metric"' gpurun_out/c4prof.log | cut -c1-200
timeout -k 10 300 python tools/shape_prof.py --top 80 > gpurun_out/shapes_c2.txt 2>&1 || { tail -5 gpurun_out/shapes_c2.txt; exit 1; }
timeout -k 10 300 python tools/shape_prof.py --model efficientdet-d4 --batch 4 --dtype bf16 --top 80 > gpurun_out/shapes_c4.txt 2>&1 || { tail -5 gpurun_out/shapes_c4.txt; exit 1; }
head -3 gpurun_out/shapes_c2.txt gpurun_out/shapes_c4.txt
