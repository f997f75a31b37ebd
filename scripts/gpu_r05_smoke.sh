# GPU: __graft_entry__.smoke() on the final tree
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke_final.log; exit $rc
