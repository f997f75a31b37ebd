# GPU: kernel traces of the fused-sepconv diagnostic builds (PHX_SEP_SKIP masks) against the real one
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for v in "" _s1 _s2 _s4 _s8; do
  PHX_CONC=0 PHX_LIB=libphx$v.so timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/kt$v -o run --output-format csv -- \
    python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/kt$v.log 2>&1 || exit 3
  echo "== libphx$v"; python tools/kt_summary.py gpurun_out/kt$v/run_kernel_trace.csv k_sep_fwd
done
