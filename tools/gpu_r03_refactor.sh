# round 3: the product / tools split (no PMENV_AB in pmenv.hip) — the GPU suite on the
# product library, then the tools library's hooks exercised through ab_libs (each variant
# must give the product's bits where it computes the same thing)
set -u
export TMPDIR=/tmp
bash tools/gpu_tests.sh r03j || exit $?
NEW=pm-rl_amd/pmenv/libpmenv.so; AB=tools/libpmenv_ab.so; PREV=tools/libpmenv_prev.so
ab() {
  timeout -k 10 300 python3 tools/ab_libs.py --libs $2 --path $3 --envs $4 --assets $5 --commission $6 \
    --reward $7 "${@:8}" > gpurun_out/ab_$1_$4x$5_c$6.json 2>> gpurun_out/ab_r03rf.err || { tail -5 gpurun_out/ab_r03rf.err; exit 1; }
}
ab rf $PREV,$NEW,$AB,$AB+PMENV_FLAT1_GEOM=256x4,$AB+PMENV_FLAT1_POL=6,$AB+PMENV_FLAT1_XCD=1 flat,flat,flat,flat,flat,flat 65536 30 0 log_returns --rounds 3 --steps 10
ab rf $NEW,$AB+PMENV_K1=reg,$AB+PMENV_STREAM_POL=2,$AB+PMENV_FLAT_IP_BLOCK=256+PMENV_FLAT_IP_VEC=4,$AB+PMENV_K1=reg+PMENV_K1_GROUPS=2 two_launch,two_launch,two_launch,two_launch,two_launch 16384 30 0 log_returns --rounds 3
ab rfo $NEW,$AB+PMENV_K1=reg+PMENV_FLAT_DB_WG=0,$AB+PMENV_ONE_V=8,$AB+PMENV_K1=reg+PMENV_FUSED=all two_launch,two_launch,one_launch,auto 4096 30 0 log_returns --rounds 3 --out
ab rf $NEW,$AB+PMENV_FLAT1_GEOM=128x8,$AB+PMENV_ONE_NOCAP=1 flat,flat,auto 2048 100 0 log_returns --rounds 3
timeout -k 10 300 python3 tools/ab_libs.py --libs $NEW,$AB+PMENV_ABLATE=129,$AB+PMENV_ABLATE=65+PMENV_K1=reg --path one_launch,one_launch,two_launch --envs 4096 --assets 30 --rounds 3 > gpurun_out/ab_rfabl.json 2>> gpurun_out/ab_r03rf.err || exit 1
grep "^#" gpurun_out/ab_r03rf.err
