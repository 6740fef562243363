# round 3: the in-place flat stream without its LDS image (direct shifted loads), and the
# side-data ablation of both forms, against the product two-launch step (tools build)
set -u
export TMPDIR=/tmp
TAG=${1:-r03d}
mkdir -p gpurun_out
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
ab() {  # envs assets rounds steps
  timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$AB+PMENV_FLAT_DIRECT=1,$AB+PMENV_ABLATE=79,$AB+PMENV_FLAT_DIRECT=1+PMENV_FLAT_DIRECT_ABL=15 \
    --path two_launch,two_launch,two_launch,two_launch --envs $1 --assets $2 --rounds $3 --steps $4 \
    > gpurun_out/ab_direct_${TAG}_$1x$2.json 2>> gpurun_out/ab_direct_$TAG.err || { tail -5 gpurun_out/ab_direct_$TAG.err; exit 1; }
}
ab 8192 30 7 40
ab 4096 30 7 40
ab 16384 30 5 20
ab 65536 30 3 10
ab 8192 16 7 40
grep "^#" gpurun_out/ab_direct_$TAG.err
