# GPU: kernel stats of the C2 step with the expand->dw fusion on and off
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for x in 1 0; do
  PHX_XDW=$x timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/xprof_$x -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/xprof_$x.log 2>&1 || { tail -20 gpurun_out/xprof_$x.log; exit 1; }
done
find gpurun_out/xprof_1 gpurun_out/xprof_0 -name "*stats*"
