#!/bin/bash
# Same-box A/B of the trio's envs per workgroup at the per-GPU shard sizes of N = 2, 4, 8 (the driver's
# 20-step shape): the default (trio_epw) against $COG_TRIO_EPW = 32 and 64, interleaved.
#     tools/epw_ab.sh TAG
set -o pipefail
O=gpurun_out/${1:-r06epw}
mkdir -p $O
for r in 1 2; do
  for n in 8192 16384 32768; do
    for e in def 32 64; do
      E=(); [ $e != def ] && E=(env COG_TRIO_EPW=$e)
      timeout -k 10 120 "${E[@]}" python bench.py --envs-total $n --steps 20 --warmup 5 --no-extras --no-cpu-baseline \
          > $O/s.json 2>/dev/null || exit 1
      python -c "import json;d=json.loads(open('$O/s.json').read().strip().splitlines()[-1]);r=d['roofline'];print('n=$n epw=$e', '%.4g' % d['value'], round(d['ms_per_step']*1e3,3), round(r['kernel_ms']*1e3,1))" >> $O/ab.txt
    done
  done
done
cat $O/ab.txt
