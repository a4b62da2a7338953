#!/bin/bash
# Multi-rank rehearsal of the bench on a one-GPU box: N ranks under torchrun, every rank on GPU 0
# (COG_DEVICE=0: the ranks share the card, so the per-rank numbers are not the 8-GPU node's), the
# driver's 20-step shape.
#     tools/gpu_scale_rehearsal.sh TAG
set -o pipefail
OUT=gpurun_out/$1
mkdir -p "$OUT"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > "$OUT/n1.json" 2> "$OUT/n1.err" || exit 1
for n in 2 4; do
  COG_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29600 + n)) bench.py --gpus $n --steps 20 --warmup 5 > "$OUT/n$n.json" 2> "$OUT/n$n.err" || exit 1
done
for n in 1 2 4; do
  python -c "import json;d=json.loads(open('$OUT/n$n.json').read().strip().splitlines()[-1]);print('N=$n value %.4g ms/step %.4f per-gpu envs %d' % (d['value'], d['ms_per_step'], d['config']['n_envs_per_gpu']))"
done
