# GPU (round 6, closing): kernel trace of the default C2 bench command (its GEMM average must agree
# with the line's roofline.avg_us), the PMC traffic passes, the C4 and C5 lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-r06f}
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_kt -o run --output-format csv -- \
  python bench.py --no-cpu-baseline --no-secondary > gpurun_out/${tag}_kt_bench.json 2> gpurun_out/${tag}_kt.log || exit 3
f=$(find gpurun_out/${tag}_kt -name '*kernel_trace.csv' | head -1); s=$(find gpurun_out/${tag}_kt -name '*kernel_stats.csv' | head -1)
cp "$s" gpurun_out/${tag}_kernel_stats_c2.csv
python - "$f" gpurun_out/${tag}_kt_bench.json <<'PY'
import csv, json, sys
rows = list(csv.DictReader(open(sys.argv[1])))
g = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows if "k_gemm" in r["Kernel_Name"]]
d = json.load(open(sys.argv[2]))
print(f"kernel trace: {len(rows)} launches, GEMM kernels {len(g)} launches avg {sum(g) / len(g) / 1e3:.2f} us;"
      f" bench line roofline avg_us {d['roofline']['avg_us']} over {d['roofline']['launches']} launches/step")
PY
rm -rf gpurun_out/${tag}_kt
bash scripts/gpu_pmc.sh > gpurun_out/${tag}_pmc.log 2>&1 || { tail -3 gpurun_out/${tag}_pmc.log; exit 3; }
python scripts/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/${tag}_pmc_traffic.json detector "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), python bench.py --steps 2 --warmup 1 (C2, round 6)" > gpurun_out/${tag}_pmc_summary.txt 2>&1 || exit 3
tail -12 gpurun_out/${tag}_pmc_summary.txt
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 300 python bench.py --model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16 --steps 30 --no-secondary > gpurun_out/${tag}_bench_d4bf16.json 2> gpurun_out/${tag}_bench_d4bf16.err || exit 3
python -c "import json;d=json.load(open('gpurun_out/${tag}_bench_d4bf16.json'));print('C4', d['ms_per_step'], d['value'], d['roofline']['frac'])"
timeout -k 10 300 python tools/defender_bench.py > gpurun_out/${tag}_defender.json 2> gpurun_out/${tag}_defender.err || exit 3
python -c "import json;d=json.load(open('gpurun_out/${tag}_defender.json'));print('C5', d['ms_per_step'], d['value'], d['roofline'] is not None, d['cpu_baseline'] is not None)"
