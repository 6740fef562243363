# round 4: the batched reward's bit fingerprints from the library of record
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/f2_bits.py > gpurun_out/f2_bits.json 2> gpurun_out/f2_bits.err || { tail -5 gpurun_out/f2_bits.err; exit 1; }
wc -l gpurun_out/f2_bits.json
timeout -k 10 120 ./tools/exp_check > gpurun_out/exp_check.log 2>&1; echo "exp_check rc=$?"; cat gpurun_out/exp_check.log
