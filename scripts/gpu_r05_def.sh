# GPU: C5 defender line + kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/defender_bench.py --no-cpu-baseline > gpurun_out/def_bench.json 2> gpurun_out/def_bench.err || { tail -5 gpurun_out/def_bench.err; exit 1; }
cut -c1-400 gpurun_out/def_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/defprof -o run --output-format csv -- python3 tools/defender_bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-profile > gpurun_out/defprof.log 2>&1 || { tail -20 gpurun_out/defprof.log; exit 1; }
