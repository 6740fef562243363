# round 4: the f2 forward in one launch with an epoch-tagged ticket and no fence (tools build,
# PMENV_BR_TICKET) against the product's two launches, bits compared
set -u
export TMPDIR=/tmp
TAG=${1:-r04y}
mkdir -p gpurun_out
timeout -k 10 300 python3 pm-rl_amd/build.py --ab-only > gpurun_out/build_ab_$TAG.log 2>&1 || { tail -5 gpurun_out/build_ab_$TAG.log; exit 1; }
timeout -k 10 300 python3 tools/ab_f2.py --knobs PMENV_BR_TICKET=1 --shapes 65536x30,16384x30,4096x30,65536x64,1000x7 \
  > gpurun_out/ab_f2t_$TAG.json 2> gpurun_out/ab_f2t_$TAG.err || { tail -5 gpurun_out/ab_f2t_$TAG.err; exit 1; }
timeout -k 10 300 python3 tools/ab_f2.py --knobs PMENV_BR_TICKET=1 --shapes 65536x30,4096x30 --kind sharpe_ratio \
  > gpurun_out/ab_f2ts_$TAG.json 2>> gpurun_out/ab_f2t_$TAG.err || { tail -5 gpurun_out/ab_f2t_$TAG.err; exit 1; }
grep "^#" gpurun_out/ab_f2t_$TAG.err
