# round 4: what bounds the f2 forward's rows kernel: kernel trace, then a PMC pass of VALU
# issue counters (SQ_ACTIVE_INST_VALU / SQ_BUSY_CYCLES / SQ_WAVE_CYCLES per dispatch)
set -u
export TMPDIR=/tmp
TAG=${1:-r04n}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/f2k_$TAG -o run --output-format csv -- \
  python3 tools/f2_pmc.py --calls 20 > gpurun_out/f2k_$TAG.log 2>&1 || { tail -5 gpurun_out/f2k_$TAG.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE \
  -d gpurun_out/f2p_$TAG -o run --output-format csv -- python3 tools/f2_pmc.py --calls 5 > gpurun_out/f2p_$TAG.log 2>&1 || { tail -5 gpurun_out/f2p_$TAG.log; exit 1; }
grep -E "batch_reward" gpurun_out/f2k_$TAG/run_kernel_stats.csv | cut -c1-160
