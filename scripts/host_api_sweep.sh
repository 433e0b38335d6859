set -u
cd $GRAFT_REPO_ROOT
for t in 4 8 16; do for c in 0 8 64; do
echo "threads=$t chunk_mb=$c $(SWBANK_HOST_THREADS=$t SWBANK_CHUNK_MB=$c timeout -k 10 120 python scripts/host_api_bench.py --iters 5)"
done; done
timeout -k 10 60 python - <<'PY'
import torch, time
x = torch.empty(142*2**20, dtype=torch.uint8).pin_memory(); d = torch.empty_like(x, device='cuda')
for _ in range(3): d.copy_(x, non_blocking=True)
torch.cuda.synchronize(); t=time.perf_counter()
for _ in range(10): d.copy_(x, non_blocking=True)
torch.cuda.synchronize(); print("pinned H2D GB/s", 10*x.numel()/(time.perf_counter()-t)/1e9)
PY
nproc
