# A/B of tile-kernel variants on protein shapes (scratch tuning script)
set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in 1 2; do
for r in 16 32; do
echo R=$r
SWBANK_R=$r timeout -k 10 300 python scripts/wave_sweep.py --kernel tile --qlen 128 --L 300 --ns 131072 --wpb 4 || exit 3
SWBANK_R=$r timeout -k 10 300 python scripts/wave_sweep.py --kernel tile --qlen 256 --L 300 --ns 65536 --wpb 4 || exit 3
SWBANK_R=$r timeout -k 10 300 python scripts/wave_sweep.py --kernel tile --qlen 512 --L 300 --ns 65536 --wpb 4 || exit 3
done; done
