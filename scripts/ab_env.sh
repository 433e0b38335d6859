# A/B of an environment knob on the headline bench (scratch tuning):
#   AB_VAR=SWBANK_ROTATE AB_VALS="0 1" bash scripts/ab_env.sh
set -u
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
for v in ${AB_VALS}; do
env $AB_VAR=$v timeout -k 10 300 python bench.py --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/ab.json || exit 3
python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$AB_VAR=$v', d['value'], d['roofline']['kernel_gcups'], d['kernel'])"
done; done
