#!/bin/bash
# Same-box A/B of the trio's form at the driver's shape (65,536 envs): the two-per-CU form (default
# above one workgroup per CU) against the LAT form ($COG_TRIO_JT=1) and three workgroups per CU ($COG_TRIO_WPC=3),
# interleaved.      tools/jt_ab.sh TAG
set -o pipefail
O=gpurun_out/${1:-r06jt}
mkdir -p $O
line() { python -c "import json,sys;d=json.loads(open('$1').read().strip().splitlines()[-1]);r=d['roofline'];print('$2', '%.4g' % d['value'], round(d['ms_per_step']*1e3,3), round(r['kernel_ms']*1e3,1))"; }
for r in 1 2; do
  for jt in def 1 w3; do
    E=(); [ $jt = 1 ] && E=(env COG_TRIO_JT=1); [ $jt = w3 ] && E=(env COG_TRIO_WPC=3)
    timeout -k 10 120 "${E[@]}" python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $O/d_$jt.json 2>/dev/null || exit 1
    line $O/d_$jt.json "jt=$jt 20-step " >> $O/ab.txt
    timeout -k 10 120 "${E[@]}" python bench.py --steps 2000 --warmup 200 --no-extras --no-cpu-baseline > $O/k_$jt.json 2>/dev/null || exit 1
    line $O/k_$jt.json "jt=$jt 1000-step" >> $O/ab.txt
  done
done
cat $O/ab.txt
