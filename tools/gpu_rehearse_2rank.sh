# Two ranks sharing the one GPU over gloo (RCCL refuses two ranks on one device): the
# multi-rank bench path (weak and strong scaling) on the product step; then the default
# bench twice more (kernel-time spread, slowest sample).
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --steps 50 --warmup 5 --dist-backend gloo \
    > gpurun_out/bench_2rank_rehearsal_$TAG.json 2> gpurun_out/bench_2rank_rehearsal_$TAG.err || exit $?
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29512 bench.py --gpus 2 --global-envs 65536 --steps 50 --warmup 5 --dist-backend gloo \
    > gpurun_out/bench_2rank_strong_$TAG.json 2> gpurun_out/bench_2rank_strong_$TAG.err || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 > gpurun_out/bench_rep${i}_$TAG.json 2> gpurun_out/bench_rep${i}_$TAG.err || exit $?
done
