# GPU: guard bands after every executor allocation (PHX_GUARD_BYTES) around C4 (D4 bf16 1024^2 x 4)
# and C2 steps: any write past a buffer's end is reported on stderr after the step.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  tag=$1; shift
  timeout -k 10 300 env PHX_GUARD_BYTES=1048576 "$@" python bench.py --no-cpu-baseline --no-profile --no-secondary --steps 3 --warmup 1 $BARGS > gpurun_out/guard_$tag.json 2> gpurun_out/guard_$tag.err
  rc=$?; echo "$tag rc=$rc guard reports: $(grep -c 'phx guard' gpurun_out/guard_$tag.err)"; grep 'phx guard' gpurun_out/guard_$tag.err | sort | uniq -c | head -20
  return $rc
}
BARGS="--model efficientdet-d4 --dtype bf16 --image-size 1024 --batch 4"
run d4_default && run d4_early PHX_FORK_FRAC=0.2 && run d4_onestream PHX_CONC=0 && \
BARGS="" run c2_default && BARGS="--model efficientdet-d4 --image-size 1024 --batch 4" run d4f32_early PHX_FORK_FRAC=0.2
