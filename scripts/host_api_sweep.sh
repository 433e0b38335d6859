# host-buffer feeder sweep: 2-bit packing x worker threads x chunk size (scratch tuning script)
set -u
cd $GRAFT_REPO_ROOT
for p in 1 0; do for t in 8 16; do for c in 0 4 16; do
echo "pack2=$p threads=$t chunk_mb=$c $(SWBANK_PACK2=$p SWBANK_HOST_THREADS=$t SWBANK_CHUNK_MB=$c timeout -k 10 120 python scripts/host_api_bench.py --iters 10)"
done; done; done
