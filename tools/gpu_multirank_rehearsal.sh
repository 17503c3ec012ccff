# GPU run: rehearse bench.py's N > 1 control flow (export_depth + all_gather + max-over-ranks timing)
# with 2 ranks on the box's one GPU over gloo (RCCL needs one GPU per rank; the driver's 8-GPU node
# runs the real "nccl" path).  Log under gpurun_out/.
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
DPE_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --no-pass-types \
  > gpurun_out/${1:-r02}_multirank.log 2>&1
rc=$?
echo "multirank rc=$rc" >> gpurun_out/${1:-r02}_multirank.log
exit $rc
