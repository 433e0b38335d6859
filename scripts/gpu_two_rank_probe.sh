#!/bin/bash
# Two bench ranks sharing the box's GPU (gloo), with environment settings per run:
#   ENVS="A=1|-" [W=q100xdata500] [REPS=64] [STEPS=3] bash scripts/gpu_two_rank_probe.sh
# prints each run's parity_sample; outputs gpurun_out/tr_<i>.json
set -u
cd ${GRAFT_REPO_ROOT:-$(dirname "$0")/..}
mkdir -p gpurun_out
IFS='|' read -ra E <<< "$ENVS"
for i in "${!E[@]}"; do
  ev=""; [ "${E[$i]}" != "-" ] && ev="${E[$i]}"
  port=$((29500 + RANDOM % 1000))
  env $ev SWBENCH_BACKEND=gloo SWBENCH_SHARE_GPU=1 MASTER_ADDR=127.0.0.1 timeout -k 10 240 \
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus 2 --steps ${STEPS:-3} --warmup 1 --reps ${REPS:-64} \
    --cpu-seconds 0 --workload ${W:-q100xdata500} > gpurun_out/tr_$i.json 2> gpurun_out/tr_$i.err
  rc=$?; [ $rc -eq 0 ] || { echo "${E[$i]} rc=$rc"; tail -5 gpurun_out/tr_$i.err; exit $rc; }
  python3 -c "import json,sys; l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d=json.loads(l); print(sys.argv[2], d['kernel'][-40:], d['parity_sample'])" gpurun_out/tr_$i.json "${E[$i]}"
done
