# GPU: kernel-trace profiles of the bench under several environment settings (per-kernel A/B).
# usage: bash scripts/gpu_prof_ab.sh "ENV=.." "ENV=.." ...   -> gpurun_out/profab<i>/run_kernel_stats.csv
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
i=0
for setting in "$@"; do
  for kv in $setting; do export "$kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profab$i -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --steps 10 --warmup 2 --no-profile > gpurun_out/profab$i.log 2>&1
  rc=$?; echo "[$setting] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  for kv in $setting; do unset "${kv%%=*}"; done
  i=$((i+1))
done
