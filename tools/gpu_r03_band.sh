# round 3: the in-place 48-256 MiB band (cache-resident windows, the per-GPU shares of the
# 8-GPU curve): two launches vs the one-workgroup-per-env step (4 / 6 / 8 chunks per lane)
# vs the flat step, in-process interleaved, on the final product kernels
set -u
export TMPDIR=/tmp
TAG=${1:-r03u}
mkdir -p gpurun_out
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
ab() {  # envs assets rounds steps
  timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$L,$AB+PMENV_ONE_V=6,$AB+PMENV_ONE_V=8,$L \
    --path two_launch,one_launch,one_launch,one_launch,flat --envs $1 --assets $2 --rounds $3 --steps $4 \
    > gpurun_out/ab_band_${TAG}_$1x$2.json 2>> gpurun_out/ab_band_$TAG.err || { tail -5 gpurun_out/ab_band_$TAG.err; exit 1; }
}
ab 1536 30 9 40
ab 2048 30 9 40
ab 3072 30 9 40
ab 4096 30 9 40
ab 6144 30 7 40
ab 8192 30 7 40
ab 4096 16 9 40
ab 8192 16 7 40
ab 2048 64 9 40
ab 4096 64 7 40
ab 8192 8 7 40
ab 16384 8 7 40
ab 3072 32 9 40
grep "^#" gpurun_out/ab_band_$TAG.err
