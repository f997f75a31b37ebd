# GPU (one card): rehearsal of bench.py's N=2 path — two ranks on cuda:0 over gloo (RCCL needs one GPU
# per rank), the driver's torch.distributed.run launch line, max-over-ranks timing, one JSON line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
PHX_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/dp2.json 2> gpurun_out/dp2.err
rc=$?; echo "dp2 rc=$rc"; cat gpurun_out/dp2.json; tail -3 gpurun_out/dp2.err
