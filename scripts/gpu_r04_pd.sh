# GPU: GEMM prefetch depth (PHX_GEMM_PD 1-4 libraries) per shape with tools/gemm_bench, modes 0 / 1 / 3,
# then the C2 step with each library (bench.py, PHX_LIB).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "" _pd2 _pd3 _pd4; do
  d=/tmp/lib$v; mkdir -p $d; ln -sf "$PWD/mladversarialobjectdetection_amd/libphx$v.so" $d/libphx.so
  for m in 0 1 3; do
    GEMM_MODE=$m LD_LIBRARY_PATH=$d timeout -k 10 120 ./tools/gemm_bench > gpurun_out/pd$v.m$m.txt 2>&1
    rc=$?; echo "lib$v mode $m rc=$rc $(grep total gpurun_out/pd$v.m$m.txt)"; [ $rc -eq 0 ] || exit $rc
  done
done
for r in 1 2; do
  for v in "" _pd2 _pd3 _pd4; do
    PHX_LIB=libphx$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-profile --no-secondary --steps 100 > gpurun_out/ab.json 2> gpurun_out/ab.err
    rc=$?; echo "c2 lib$v rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/ab.json'));print(d['ms_per_step'],d['value'])")"
    [ $rc -eq 0 ] || exit $rc
  done
done
