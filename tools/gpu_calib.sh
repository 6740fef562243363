# Same-box calibration: plain-copy ceiling (random data) next to the step A/B and the
# BASELINE configs, so ratios are not box-to-box comparisons
set -u
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -o gpurun_out/copybench tools/copybench.hip || exit 1
timeout -k 10 200 ./gpurun_out/copybench 1967 1 > gpurun_out/calib_copy.log 2>&1 || exit 1
head -3 gpurun_out/calib_copy.log; grep -E "chunk 256x1 l0|chunk 256x2 l3 s3|read 256x2 l2|write 256x2 s0" gpurun_out/calib_copy.log
ROUNDS=9 bash tools/gpu_ab_pol.sh "stream,o,stream+PMENV_FLAT_INPLACE=0" || exit 1
bash tools/bench_configs.sh
