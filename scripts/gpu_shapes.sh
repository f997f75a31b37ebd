set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/shape_prof.py --top 80 > gpurun_out/shapes_d0.txt 2>&1; echo "d0 rc=$?"
timeout -k 10 300 python tools/shape_prof.py --model efficientdet-d4 --batch 4 --dtype bf16 --top 60 > gpurun_out/shapes_d4.txt 2>&1; echo "d4 rc=$?"
