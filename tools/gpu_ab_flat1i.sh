# step_flat_kernel: split cache policies of the window stream (nt loads only / nt stores
# only) against nt for both (the product above 256 MiB), in place and double-buffered.
set -u
TAG=${1:-r02}
export TMPDIR=/tmp
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
V="stream,stream+PMENV_FLAT1_POL=5,stream+PMENV_FLAT1_POL=6,stream+PMENV_FLAT1_POL=7"
VO="o,o+PMENV_FLAT1_POL=5,o+PMENV_FLAT1_POL=6,o+PMENV_FLAT1_POL=7"
timeout -k 10 300 python tools/ab_advance.py --envs 65536 --steps 100 --rounds 9 --variants "$V" > $OUT/flat1i_ip.json 2> $OUT/flat1i_ip.err || exit 1
timeout -k 10 300 python tools/ab_advance.py --envs 65536 --steps 100 --rounds 9 --variants "$VO" > $OUT/flat1i_db.json 2> $OUT/flat1i_db.err || exit 1
