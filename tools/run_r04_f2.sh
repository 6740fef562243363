# round 4: (1) the f2 forward in one launch with epoch flags (tools build, PMENV_BR_RELAY)
# against the product's two launches; (2) the exact kernel combination of the 16,384 x 30
# leg that faulted in r03d (the tools build's default packed scalar step with its halo copy
# + the product's 512 x 2 in-place stream, and the same without the halo copy), attributed
set -u
export TMPDIR=/tmp
TAG=${1:-r04f}
mkdir -p gpurun_out
timeout -k 10 300 python3 pm-rl_amd/build.py --ab-only > gpurun_out/build_ab_$TAG.log 2>&1 || { tail -5 gpurun_out/build_ab_$TAG.log; exit 1; }
timeout -k 10 300 python3 tools/ab_f2.py --knobs PMENV_BR_RELAY=1 --shapes 65536x30,16384x30,4096x30,65536x64 \
  > gpurun_out/ab_f2_$TAG.json 2> gpurun_out/ab_f2_$TAG.err || { tail -5 gpurun_out/ab_f2_$TAG.err; exit 1; }
timeout -k 10 300 python3 tools/ab_f2.py --knobs PMENV_BR_RELAY=1 --shapes 65536x30,4096x30 --kind sharpe_ratio \
  > gpurun_out/ab_f2s_$TAG.json 2>> gpurun_out/ab_f2_$TAG.err || { tail -5 gpurun_out/ab_f2_$TAG.err; exit 1; }
grep "^#" gpurun_out/ab_f2_$TAG.err
L=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so
timeout -k 10 300 python3 tools/ab_libs.py --attribute --libs $L,$AB,$AB+PMENV_ABLATE=79 \
  --path two_launch,two_launch,two_launch --envs 16384 --assets 30 --rounds 5 --steps 20 \
  > gpurun_out/ab_r03d_repro_$TAG.json 2> gpurun_out/ab_r03d_repro_$TAG.err
rc=$?
grep "^#" gpurun_out/ab_r03d_repro_$TAG.err
exit $rc
