# GPU (timing only, wrong results): upper bounds of C2 launch kinds and of the stage 2-3 blocks
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
run() { PHX_SKIP_KINDS="$2" timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-profile > gpurun_out/skip2.json 2>/dev/null || exit 1
  echo "$1: $(python -c "import json;d=json.load(open('gpurun_out/skip2.json'));print(d['ms_per_step'])")"; }
run none ""
run fgemm "f:gemm"
run bgemm "b:gemm"
run fdw "f:dw_fwd"
run bdw "b:dw_bwd"
run fse "f:se_fwd"
run bse "b:se_bwd"
run fother "f:fwd_other"
run bother "b:bwd_other"
run bbnred "b:bn_bwd_reduce"
run blk123 "|blocks_1/,blocks_2/,blocks_3/"
run blk1exp "|blocks_1/conv2d,blocks_1/tpu_batch_normalization,blocks_1/depthwise"
run none2 ""
