# round 3: the flat stream's side data (bar rows, w') staged in LDS per wave against the
# per-chunk selects from scalar registers (tools build twin), in place and double-buffered
set -u
export TMPDIR=/tmp
TAG=${1:-r03l}
mkdir -p gpurun_out
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so; B=tools/libpmenv_base.so
ab() {  # envs assets rounds steps [--out]
  timeout -k 10 300 python3 tools/ab_libs.py --libs $L,$AB+PMENV_FLAT_SSEL=1+PMENV_K1=reg,$AB+PMENV_K1=reg --path two_launch,two_launch,two_launch --envs $1 --assets $2 \
    --rounds $3 --steps $4 "${@:5}" > gpurun_out/ab_lside_${TAG}_$1x$2.json 2>> gpurun_out/ab_lside_$TAG.err || { tail -5 gpurun_out/ab_lside_$TAG.err; exit 1; }
}
ab 8192 30 9 40
ab 4096 30 9 40
ab 8192 16 9 40
ab 16384 8 9 40
ab 65536 30 3 10
ab 4096 30 7 40 --out
grep "^#" gpurun_out/ab_lside_$TAG.err
