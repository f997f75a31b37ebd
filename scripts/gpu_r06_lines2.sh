# GPU (round 6, closing): the C4 and C5 lines, and the C2 line once more (profile report fix)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
tag=${1:-r06g}
timeout -k 10 300 python bench.py --model efficientdet-d4 --image-size 1024 --batch 4 --dtype bf16 --steps 30 --no-secondary > gpurun_out/${tag}_bench_d4bf16.json 2> gpurun_out/${tag}_bench_d4bf16.err || { grep -v amdgpu gpurun_out/${tag}_bench_d4bf16.err | tail -5; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/${tag}_bench_d4bf16.json'));print('C4', d['ms_per_step'], d['value'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['traffic'])"
timeout -k 10 300 python tools/defender_bench.py > gpurun_out/${tag}_defender.json 2> gpurun_out/${tag}_defender.err || { tail -5 gpurun_out/${tag}_defender.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/${tag}_defender.json'));print('C5', d['ms_per_step'], d['value'], d['roofline'] is not None, d['cpu_baseline'] is not None)"
