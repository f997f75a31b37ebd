# GPU: the forward EOT resize over XCD bands of row tiles (k_eot_bands + k_eot_resize) against the
# previous build (libphx_prev.so): whole steps bit for bit (attacker, both placement flows; defender),
# the EOT / parity suites, alternating A/B of the reference's placement flow (first-pass boxes) and C2
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-eotb}
for L in libphx_prev.so libphx.so; do
  PHX_LIB=$L timeout -k 10 300 python tools/step_hash.py > gpurun_out/${tag}_hash_$L.txt 2>&1 || exit 3
  PHX_LIB=$L timeout -k 10 300 python tools/step_hash.py --defender >> gpurun_out/${tag}_hash_$L.txt 2>&1 || exit 3
  grep -v amdgpu.ids gpurun_out/${tag}_hash_$L.txt
done
timeout -k 10 700 python -u -m pytest tests/test_gpu_eot_v2.py tests/test_gpu_eot_edges.py tests/test_gpu_parity.py tests/test_gpu_firstpass.py -q -m gpu \
  -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/${tag}_tests.log; grep -E "^FAILED|^ERROR" gpurun_out/${tag}_tests.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for r in 1 2 3; do
  for L in libphx_prev.so libphx.so; do
    PHX_LIB=$L timeout -k 10 200 python bench.py --placement first-pass --person-bias 4.6 --steps 40 --no-cpu-baseline --no-secondary --no-profile > gpurun_out/${tag}_fp_$L.json 2>gpurun_out/${tag}_fp_$L.err || exit 3
    echo "round $r first-pass flow $L: $(python -c "import json;d=json.load(open('gpurun_out/${tag}_fp_$L.json'));print(d['ms_per_step'], d['value'])")"
  done
done
for L in libphx_prev.so libphx.so; do
  PHX_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-profile > gpurun_out/${tag}_c2_$L.json 2>gpurun_out/${tag}_c2_$L.err || exit 3
  echo "C2 $L: $(python -c "import json;d=json.load(open('gpurun_out/${tag}_c2_$L.json'));print(d['ms_per_step'])")"
done
exit $rc
