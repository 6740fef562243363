set -u
export TMPDIR=/tmp
bash tools/gpu_tests.sh r03d || exit $?
bash tools/gpu_ab_libs.sh split tools/libpmenv_base.so pm-rl_amd/pmenv/libpmenv.so auto
