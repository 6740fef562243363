# round 4: HBM-side traffic of the relayed step at config 4's 8-GPU share (8,192 x 30 in place,
# Infinity-Cache resident): FETCH_SIZE and WRITE_SIZE passes of the bench at that share
set -u
export TMPDIR=/tmp
TAG=${1:-r04za}
mkdir -p gpurun_out
ARGS="--global-envs 8192 --steps 10 --warmup 2 --cpu-baseline 0 --alt-steps 0 --parity-envs 64"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/rpf_$TAG -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/rpf_$TAG.log 2>&1 || { tail -5 gpurun_out/rpf_$TAG.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/rpw_$TAG -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/rpw_$TAG.log 2>&1 || { tail -5 gpurun_out/rpw_$TAG.log; exit 1; }
echo done
