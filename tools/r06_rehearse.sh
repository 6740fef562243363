#!/bin/bash
# Round 6: the multi-rank bench path on the final library — two ranks sharing the one GPU over
# gloo (RCCL refuses two ranks on one device), weak and strong (BASELINE config 4's 65,536 envs
# split over the ranks): tools/gpu_rehearse_2rank.sh's first two runs.
set -o pipefail
T=${1:-r06end}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 2 --steps 50 --warmup 5 --dist-backend gloo \
    > gpurun_out/bench_2rank_rehearsal_$T.json 2> gpurun_out/bench_2rank_rehearsal_$T.err || exit $?
tail -c 600 gpurun_out/bench_2rank_rehearsal_$T.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29512 bench.py --gpus 2 --global-envs 65536 --steps 50 --warmup 5 --dist-backend gloo \
    > gpurun_out/bench_2rank_strong_$T.json 2> gpurun_out/bench_2rank_strong_$T.err || exit $?
tail -c 600 gpurun_out/bench_2rank_strong_$T.json
