set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
PHX_NMS_STATS=1 timeout -k 10 200 python tools/defender_bench.py --steps 1 --warmup 0 > gpurun_out/nmsdbg_def.txt 2>&1
rc=$?; echo "def dbg rc=$rc"; grep "nms image" gpurun_out/nmsdbg_def.txt | head -12
