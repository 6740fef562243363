# GAE tile: product (72 VGPRs, 7 waves per SIMD) vs the 64-VGPR form (8 waves per SIMD:
# every workgroup of a 65,536-env rollout resident at once) vs the pipelined E = 4 tile;
# interleaved rounds in one process
set -u
mkdir -p gpurun_out
timeout -k 10 400 python3 tools/ab_gae.py --shapes 256x65536,256x131072,512x65536,256x49152,256x32768,128x65536 --rounds 9 \
  --variants "PMENV_GAE=tile+PMENV_GAE_U=8,PMENV_GAE=tile8+PMENV_GAE_U=8,PMENV_GAE=tile+PMENV_GAE_U=4+PMENV_GAE_E=4" \
  > gpurun_out/ab_gae2.json 2> gpurun_out/ab_gae2.err || { tail -20 gpurun_out/ab_gae2.err; exit 1; }
cat gpurun_out/ab_gae2.json
