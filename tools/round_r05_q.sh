# the generic stream's tile with dynamic side LDS: 256 x 4 everywhere against the product's rule
set -u
export TMPDIR=/tmp
TAG=${1:-r05q}
mkdir -p gpurun_out
PMENV_GEN_GEOM=256x4 PMENV_GEN_PERELEM=0 AB_GEN_FORCE=1 AB_R=5 timeout -k 10 400 python tools/ab_gen.py > gpurun_out/${TAG}_g4.json 2> gpurun_out/${TAG}_g4.err || { tail -5 gpurun_out/${TAG}_g4.err; exit 1; }
grep -v "^[WE]2" gpurun_out/${TAG}_g4.err | python3 -c "
import sys,json
for l in sys.stdin:
    k,_,j=l.partition(' ')
    try: o=json.loads(j)
    except Exception: continue
    print(k, round(o['gen']['us'],1), round(o['small']['us'],1), o['windows_equal'], o['rewards_equal'])
"
