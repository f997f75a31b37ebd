# GPU: C5 A/B of the wave-split-K kernel (1x1 convs and the U-Net's implicit im2col), then the mid-K sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for x in 0 1; do
    PHX_GEMM_WSK=$x timeout -k 10 300 python tools/defender_bench.py --no-cpu-baseline --no-profile > gpurun_out/wskd_$x.json 2>/dev/null || exit 1
    echo "C5 round $r PHX_GEMM_WSK=$x: $(python -c "import json;d=json.load(open('gpurun_out/wskd_$x.json'));print(d['ms_per_step'], d['value'])")"
  done
done
bash scripts/gpu_r05_wsk2.sh
