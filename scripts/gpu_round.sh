# GPU, end of a work block: parity tests -> default bench line (cpu_baseline + roofline) ->
# rocprofv3 kernel-trace summary -> PMC HBM-traffic passes (each step bounded, stop at first failure)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_all.sh || exit $?
bash scripts/gpu_pmc.sh || exit $?
