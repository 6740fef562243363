# the scalar phase with (in place: copies the flat stream's halo) and without
# (double-buffered) the halo copy
set -u
mkdir -p gpurun_out
run() {
  timeout -k 10 300 python tools/ab_advance.py --envs $2 --assets $3 --steps ${STEPS:-100} --rounds ${ROUNDS:-7} \
      --phases $4 --variants "$5" > gpurun_out/abk1h_$1.log 2> gpurun_out/abk1h_$1.err || { tail -5 gpurun_out/abk1h_$1.err; return 1; }
  python -c "
import json; t=open('gpurun_out/abk1h_$1.log').read(); d=json.loads(t[t.index('{'):])
for k,v in d['variants'].items(): print('$1', f\"{k:34s} {v['median_us']:8.2f} us  min {v['min_us']:8.2f}\")
"
}
run k1_65536 65536 30 1 "stream,o,stream+PMENV_K1=reg,o+PMENV_K1=reg" &&
run k1_8192x500 8192 500 1 "stream,o,stream+PMENV_K1=reg,o+PMENV_K1=reg" &&
run step_8192x500 8192 500 0 "stream,o"
