# round 3: the in-place 48-256 MiB band, more asset counts (two launches vs one workgroup
# per env vs the flat step), in-process interleaved
set -u
export TMPDIR=/tmp
TAG=${1:-r03w}
mkdir -p gpurun_out
L=pm-rl_amd/pmenv/libpmenv.so
ab() {  # envs assets rounds steps paths
  n=$(echo $5 | tr ',' '\n' | wc -l); libs=$(yes $L | head -$n | paste -sd,)
  timeout -k 10 300 python3 tools/ab_libs.py --libs $libs --path $5 --envs $1 --assets $2 --rounds $3 --steps $4 \
    > gpurun_out/ab_band_${TAG}_$1x$2.json 2>> gpurun_out/ab_band_$TAG.err || { tail -5 gpurun_out/ab_band_$TAG.err; exit 1; }
}
P3=two_launch,one_launch,flat
ab 2048 32 9 40 $P3
ab 3072 32 9 40 $P3
ab 4096 32 9 40 $P3
ab 4096 8 9 40 $P3
ab 8192 8 9 40 $P3
ab 16384 8 7 40 $P3
ab 3072 16 9 40 $P3
ab 6144 16 9 40 $P3
ab 2048 48 9 40 $P3
ab 4096 48 7 40 $P3
ab 1024 64 9 40 two_launch,flat
ab 2048 64 9 40 two_launch,flat
ab 4096 64 7 40 two_launch,flat
ab 2048 30 9 40 $P3
grep "^#" gpurun_out/ab_band_$TAG.err
