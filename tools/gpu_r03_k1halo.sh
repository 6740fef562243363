# round 3: the register scalar step with its halo copy loaded beside the step's loads and
# stored at the end (HaloRegs) against the previous build (copy first), two launches
set -u
export TMPDIR=/tmp
TAG=${1:-r03h2}
mkdir -p gpurun_out
B=tools/libpmenv_base.so; L=pm-rl_amd/pmenv/libpmenv.so
ab() {  # envs assets rounds steps
  timeout -k 10 300 python3 tools/ab_libs.py --libs $B,$L,$B,$L --path two_launch,two_launch,auto,auto --envs $1 --assets $2 \
    --rounds $3 --steps $4 > gpurun_out/ab_k1h_${TAG}_$1x$2.json 2>> gpurun_out/ab_k1h_$TAG.err || { tail -5 gpurun_out/ab_k1h_$TAG.err; exit 1; }
}
ab 8192 30 9 40
ab 4096 30 9 40
ab 6144 30 9 40
ab 8192 16 9 40
ab 16384 8 9 40
ab 4096 48 9 40
ab 65536 30 3 10
grep "^#" gpurun_out/ab_k1h_$TAG.err
