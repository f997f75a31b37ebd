# GPU: prefetch edge-case tests, then the closing evidence (scripts/gpu_r05_evid3.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r05_pfa3.sh && bash scripts/gpu_r05_evid3.sh
