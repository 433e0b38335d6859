# host-buffer feeder sweep: worker threads x chunk size (scratch tuning script)
set -u
cd $GRAFT_REPO_ROOT
for t in 8 16; do for c in 0 4 8 16 24; do
echo "threads=$t chunk_mb=$c $(SWBANK_HOST_THREADS=$t SWBANK_CHUNK_MB=$c timeout -k 10 120 python scripts/host_api_bench.py --iters 10)"
done; done
