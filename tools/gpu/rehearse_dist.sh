# Rehearse the driver's N>1 bench launch on a 1-GPU box: N ranks share cuda:0,
# collectives on gloo (PGW_BENCH_REHEARSE=1).  Checks the torchrun path only;
# the per-rank numbers are meaningless (ranks contend for one GPU).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
N=${1:-2}
PGW_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus $N --steps 40 --warmup 5 \
  --batch 16384 > gpurun_out/rehearse_$N.log 2>&1
rc=$?
tail -3 gpurun_out/rehearse_$N.log | cut -c1-600
exit $rc
