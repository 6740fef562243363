# The strong-scaling curve's per-GPU shares on one GPU: 65,536 global envs split over
# N = 2 / 4 / 8 ranks is 32,768 / 16,384 / 8,192 envs per GPU; each share is timed alone
# (bench.py --global-envs S at N = 1), then the driver's N = 2 form rehearsed with two
# ranks sharing the GPU over gloo (RCCL refuses two ranks on one device).
set -u
TAG=${1:-r04}
export TMPDIR=/tmp
mkdir -p gpurun_out
for S in 32768 16384 8192; do
  timeout -k 10 300 python bench.py --global-envs $S --cpu-baseline 0 \
      > gpurun_out/share_${S}_$TAG.json 2> gpurun_out/share_${S}_$TAG.err || exit $?
  tail -1 gpurun_out/share_${S}_$TAG.json | cut -c1-200
done
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29513 bench.py --gpus 2 --steps 50 --warmup 5 --dist-backend gloo \
    > gpurun_out/bench_2rank_strong_$TAG.json 2> gpurun_out/bench_2rank_strong_$TAG.err || exit $?
tail -1 gpurun_out/bench_2rank_strong_$TAG.json | cut -c1-300
