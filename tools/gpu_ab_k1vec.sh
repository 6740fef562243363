# K1 packed form (scalar_step_vec_kernel) vs the register / LDS forms: the scalar
# phase alone (in place: with the halo copy; "o": double-buffered, no halo) and the
# whole step, interleaved rounds in one process per shape.
set -u
mkdir -p gpurun_out
run() {  # tag envs assets phases variants
  timeout -k 10 300 python tools/ab_advance.py --envs $2 --assets $3 --steps ${STEPS:-100} --rounds ${ROUNDS:-7} \
      --phases $4 --variants "$5" > gpurun_out/abk1v_$1.log 2> gpurun_out/abk1v_$1.err || { tail -5 gpurun_out/abk1v_$1.err; return 1; }
  python -c "
import json; t=open('gpurun_out/abk1v_$1.log').read(); d=json.loads(t[t.index('{'):])
for k,v in d['variants'].items(): print('$1', f\"{k:34s} {v['median_us']:8.2f} us  min {v['min_us']:8.2f}\")
"
}
K="stream+PMENV_K1=reg,stream,o,stream+PMENV_K1=16x1,stream+PMENV_K1=32x2s,stream+PMENV_K1=8x4"
run k1_65536 65536 30 1 "$K" &&
run k1_16384 16384 30 1 "$K" &&
run k1_8192x500 8192 500 1 "stream+PMENV_K1=reg,stream,o,o+PMENV_K1=reg" &&
run step_65536 65536 30 0 "stream+PMENV_K1=reg,stream" &&
run step_8192x500 8192 500 0 "stream+PMENV_K1=reg,stream"
