set -o pipefail
mkdir -p gpurun_out/r05_s27
V=rasr_amd/lib/variants; P=rasr_amd/lib/librasr_gmm.so; O=gpurun_out/r05_s27
timeout -k 10 400 python scripts/ab_bench.py --mode fp32 --frames 32768 --rounds 6 --steps 20 $P $V/librasr_gmm_finold.so > $O/fp32.txt 2>&1 || exit $?
cat $O/fp32.txt
timeout -k 10 400 python scripts/ab_bench.py --mode fp32 --dim 45 --frames 32768 --rounds 6 --steps 20 $P $V/librasr_gmm_finold.so > $O/fp32_d45.txt 2>&1 || exit $?
cat $O/fp32_d45.txt
