# The BASELINE.json configs on one GPU through bench.py (config 4's per-GPU share = 8192 envs).
set -u
TAG=${1:-r02}
mkdir -p gpurun_out/configs_$TAG
run() { name=$1; shift; timeout -k 10 600 python bench.py "$@" > gpurun_out/configs_$TAG/cfg_$name.json 2> gpurun_out/configs_$TAG/cfg_$name.err || return $?; python -c "
import json; d=json.loads(open('gpurun_out/configs_$TAG/cfg_$name.json').read().strip().splitlines()[-1]); rf=d['roofline']
print('$name', 'lib', d['library']['sha256'][:16], 'src', (d['library']['src_sha256'] or '')[:16], f\"{d['value']/1e6:.1f}M env-steps/s\", f\"{d['ms_per_step']:.4f} ms\", f\"{rf['kernel']} {rf['kernel_us']['median']:.1f} us frac {rf['frac']:.3f} step {rf['frac_step']:.3f}\", 'l3_resident', rf['l3_resident'], 'mae', d['reward_mae'], 'cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value']/1e6,2))" | tee -a gpurun_out/configs_$TAG/summary.txt; }
run c2_4096x30 --envs-per-gpu 4096 --steps 200 --warmup 20 &&
run c3_16384x30 --envs-per-gpu 16384 --steps 200 --warmup 20 &&
run c4share_8192x30 --envs-per-gpu 8192 --steps 200 --warmup 20 &&
run c5_8192x500_dsharpe --envs-per-gpu 8192 --assets 500 --reward diff_sharpe --steps 50 --warmup 5 --parity-envs 512 --cpu-sample-envs 1024 &&
run c2_commission --envs-per-gpu 65536 --commission 0.0025 --steps 100 --warmup 10 &&
run c1_1x5 --envs-per-gpu 1 --assets 5 --steps 200 --warmup 20 --alt-steps 20
