cd $GRAFT_REPO_ROOT
for cfg in "SWBANK_WAVE_SPLIT=0" "SWBANK_WAVE_SPLIT=100000 SWBANK_WAVE_SPLIT_P=2" "SWBANK_WAVE_SPLIT=100000 SWBANK_WAVE_SPLIT_P=4"; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python scripts/wave_sweep.py --ns 256,512,1024,2048,4096 --wpb 4 --iters 10 2>&1 | grep qlen || exit 1
  env $cfg timeout -k 10 200 python scripts/wave_sweep.py --qlen 300 --L 300 --ns 512,1024,2048,4096 --wpb 4 --iters 10 2>&1 | grep qlen || exit 1
done
