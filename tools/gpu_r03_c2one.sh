# round 3: the one-launch kernels (step_flat_kernel, step_env_kernel, step_flat_vec_kernel)
# with the two-level compose against the previous library (per-element compose there)
set -u
export TMPDIR=/tmp
TAG=${1:-r03c2}
mkdir -p gpurun_out
B=tools/libpmenv_base.so; L=pm-rl_amd/pmenv/libpmenv.so
ab() {  # paths envs assets rounds steps extra
  timeout -k 10 300 python3 tools/ab_libs.py --libs $B,$L --path $1 --envs $2 --assets $3 --rounds $4 --steps $5 "${@:6}" \
    > gpurun_out/ab_c2_${TAG}_$2x$3.json 2>> gpurun_out/ab_c2_$TAG.err || { tail -5 gpurun_out/ab_c2_$TAG.err; exit 1; }
}
ab flat 65536 30 7 10
ab flat 65536 30 5 10 --out
ab flat 65536 30 5 10 --commission 0.0025
ab flat 16384 30 7 20
ab one_launch 4096 30 9 40
ab one_launch 2048 30 9 40
ab flat 4096 16 9 40
ab flat 16384 100 5 10
ab one_launch 65536 30 5 10
grep "^#" gpurun_out/ab_c2_$TAG.err
