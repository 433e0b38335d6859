cd $GRAFT_REPO_ROOT
for cfg in "SWBANK_AVX2=0" "SWBANK_AVX2=1"; do
env $cfg timeout -k 10 300 python -u -m pytest tests/test_gpu_feeder.py -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "many_chunks" 2>&1 | tail -6
done
