# GPU (timing only, wrong results): what removing launch kinds would be worth on C2 — forward BN
# finalizes (f), backward ones (b), both, the SE forward (s).  Alternating, two rounds.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for r in 1 2; do
  for k in none f b fb s; do
    PHX_SKIP_TIMING=$k timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-profile > gpurun_out/skip_$k.json 2>/dev/null || exit 1
    echo "round $r skip=$k: $(python -c "import json;d=json.load(open('gpurun_out/skip_$k.json'));print(d['ms_per_step'])")"
  done
done
