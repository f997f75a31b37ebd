# GPU: kernel trace of the C2 step (one stream: PHX_CONC=0, so each kernel's duration is its own),
# the per-(kernel, grid) summary and the launch count per step
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-kt}
PHX_CONC=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/kt -o run --output-format csv -- python bench.py --steps 10 --warmup 2 \
  --no-cpu-baseline --no-secondary --no-profile > gpurun_out/${tag}_kt.log 2>&1 || exit 3
f=$(find /tmp/kt -name '*kernel_trace.csv' | head -1); s=$(find /tmp/kt -name '*kernel_stats.csv' | head -1)
cp "$s" gpurun_out/${tag}_kernel_stats_c2.csv
python tools/kt_summary.py "$f" > gpurun_out/${tag}_kt_summary.txt
python - "$f" > gpurun_out/${tag}_step_seq.txt <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
# one step = the launches between two consecutive k_adam... use the last 1/12 of the trace
n = len(rows)
marks = [i for i, r in enumerate(rows) if "k_image_max" in r["Kernel_Name"]]
print("launches", n, "k_image_max marks", len(marks))
if len(marks) >= 3:
    a, b = marks[-3], marks[-2]
    print("launches between the last two step marks:", b - a)
    t0 = int(rows[a]["Start_Timestamp"])
    for r in rows[a:b]:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
        print(f"{(int(r['Start_Timestamp']) - t0) / 1000:9.1f} {d:8.2f} {r['Grid_Size_X']:>8s} {r['Kernel_Name'].split('(')[0][-90:]}")
PY
head -3 gpurun_out/${tag}_step_seq.txt
