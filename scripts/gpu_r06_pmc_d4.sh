# GPU: PMC traffic of the C4 step (D4 1024^2 x 4, bf16) for its bench line's roofline.traffic
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
PMC_CMD="python bench.py --model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16 --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-secondary" \
  bash scripts/gpu_pmc.sh > gpurun_out/d4_pmc.log 2>&1 || { tail -3 gpurun_out/d4_pmc.log; exit 3; }
python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/r06_pmc_traffic_d4bf16.json detector "python bench.py --model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16 --steps 2 --warmup 1 (C4, round 6)" > gpurun_out/d4_pmc_summary.txt 2>&1 || exit 3
tail -10 gpurun_out/d4_pmc_summary.txt
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
