# A/B of two library builds (tools/ab_libs.py) over the cache-resident in-place shares,
# the BASELINE shape, commission and N > 64. Usage: gpu_ab_libs.sh TAG LIB_A LIB_B [PATHS]
set -u
TAG=$1; LA=$2; LB=$3; PATHS=${4:-auto}
mkdir -p gpurun_out
run() {  # envs assets commission reward extra...
  timeout -k 10 300 python3 tools/ab_libs.py --libs $LA,$LB --path $PATHS --envs $1 --assets $2 --commission $3 \
    --reward $4 "${@:5}" > gpurun_out/ablibs_${TAG}_$1x$2_c$3_$4.json 2>> gpurun_out/ablibs_$TAG.err || { tail -5 gpurun_out/ablibs_$TAG.err; exit 1; }
}
run 4096 30 0 log_returns
run 8192 30 0 log_returns
run 16384 30 0 log_returns
run 65536 30 0 log_returns --rounds 5 --steps 20
run 65536 30 0.0025 log_returns --rounds 5 --steps 20
run 8192 500 0 diff_sharpe --rounds 5 --steps 10
grep "^#" gpurun_out/ablibs_$TAG.err
