# round 4: the written-out f64 exp (fmath.h): the bitwise check of exp_f64 against the device
# library on the GPU, the batched reward's fingerprints against the library of record, the
# f2 kernels' times and VALU counts, config 5's step and scalar kernel
set -u
export TMPDIR=/tmp
TAG=${1:-r04o}
mkdir -p gpurun_out
bash tools/run_r04_f2bits.sh || exit 1
cp gpurun_out/f2_bits.json tests/golden/f2_bits.json
timeout -k 10 200 hipcc --offload-arch=gfx950 -O3 -std=c++17 -o gpurun_out/exp_check tools/exp_check.hip > gpurun_out/exp_build_$TAG.log 2>&1 || { tail -5 gpurun_out/exp_build_$TAG.log; exit 1; }
timeout -k 10 120 ./gpurun_out/exp_check > gpurun_out/exp_check_$TAG.log 2>&1; rc=$?; cat gpurun_out/exp_check_$TAG.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_trainer.py -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_trainer_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_trainer_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_trainer_$TAG.log
bash tools/run_r04_f2pmc.sh $TAG || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5k_$TAG -o run --output-format csv -- \
  python3 bench.py --envs-per-gpu 8192 --assets 500 --reward diff_sharpe --steps 50 --warmup 5 --parity-envs 512 --cpu-baseline 0 --alt-steps 0 \
  > gpurun_out/c5k_$TAG.json 2> gpurun_out/c5k_$TAG.err || { tail -5 gpurun_out/c5k_$TAG.err; exit 1; }
tail -1 gpurun_out/c5k_$TAG.json | cut -c1-300
grep -E "scalar_step|advance_flat" gpurun_out/c5k_$TAG/run_kernel_stats.csv | cut -c1-160
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES -d gpurun_out/c5p_$TAG -o run --output-format csv -- \
  python3 bench.py --envs-per-gpu 8192 --assets 500 --reward diff_sharpe --steps 5 --warmup 1 --parity-envs 64 --cpu-baseline 0 --alt-steps 0 \
  > gpurun_out/c5p_$TAG.json 2> gpurun_out/c5p_$TAG.err || { tail -5 gpurun_out/c5p_$TAG.err; exit 1; }
echo done
