# round 4: the BASELINE configs on one GPU (tools/bench_configs.sh) and the strong-scaling
# shares (tools/run_shares.sh) on the round's library (the relay step in AUTO)
set -u
export TMPDIR=/tmp
TAG=${1:-r04g}
bash tools/bench_configs.sh $TAG || exit $?
bash tools/run_shares.sh $TAG || exit $?
