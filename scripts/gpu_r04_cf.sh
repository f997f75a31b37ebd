# GPU: column-reduction finals with four chunks' loads in flight (libphx.so) against the previous
# build (libphx_base.so), alternating on C2 and C4, then the round-4 final evidence.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in _base ""; do
    PHX_LIB=libphx$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --no-secondary --steps 100 > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?; echo "c2 lib$v rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
for r in 1 2; do
  for v in _base ""; do
    PHX_LIB=libphx$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --no-secondary --steps 30 --model efficientdet-d4 --dtype bf16 --image-size 1024 --batch 4 > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?; echo "c4 lib$v rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
bash scripts/gpu_r04_final.sh
