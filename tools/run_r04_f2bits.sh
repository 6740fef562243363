# round 4: the batched reward's bit fingerprints from the library of record (tools/libpmenv_r04l.so, a copy
# of the r04l build kept for the r04o run and removed after it: the product rebuilt to the same binary;
# the r04l build) and the in-tree library checked against them; exp_f64 against the device library
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/f2_bits.py --lib tools/libpmenv_r04l.so > gpurun_out/f2_bits.json 2> gpurun_out/f2_bits.err || { tail -5 gpurun_out/f2_bits.err; exit 1; }
timeout -k 10 300 python3 tools/f2_bits.py --check gpurun_out/f2_bits.json 2>> gpurun_out/f2_bits.err; echo "f2 check rc=$?"
timeout -k 10 300 python3 tools/step_bits.py --lib tools/libpmenv_r04l.so > gpurun_out/step_bits.json 2> gpurun_out/step_bits.err || { tail -5 gpurun_out/step_bits.err; exit 1; }
timeout -k 10 300 python3 tools/step_bits.py --check gpurun_out/step_bits.json 2>> gpurun_out/step_bits.err; echo "step check rc=$?"
