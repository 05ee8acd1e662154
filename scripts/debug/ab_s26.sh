set -o pipefail
mkdir -p gpurun_out/r05_s26
V=rasr_amd/lib/variants; P=rasr_amd/lib/librasr_gmm.so; O=gpurun_out/r05_s26
timeout -k 10 300 python scripts/ab_bench.py --mode fp32 --frames 32768 --rounds 3 --steps 20 $P $V/librasr_gmm_noconst.so $V/librasr_gmm_finold.so > $O/fp32.txt 2>&1 || exit $?
cat $O/fp32.txt
timeout -k 10 300 python scripts/ab_bench.py --mode fp32 --dim 45 --frames 32768 --rounds 3 --steps 20 $P $V/librasr_gmm_finold.so > $O/fp32_d45.txt 2>&1 || exit $?
cat $O/fp32_d45.txt
timeout -k 10 300 python scripts/ab_bench.py --mode simds --frames 32768 --rounds 3 --steps 20 $P $V/librasr_gmm_finold.so > $O/simds.txt 2>&1 || exit $?
cat $O/simds.txt
timeout -k 10 300 python scripts/ab_bench.py --mode simd --frames 32768 --rounds 3 --steps 20 $P $V/librasr_gmm_finold.so > $O/simd.txt 2>&1 || exit $?
cat $O/simd.txt
timeout -k 10 300 python scripts/ab_bench.py --mode sum --frames 32768 --rounds 2 --steps 10 $P $V/librasr_gmm_finold.so > $O/sum.txt 2>&1 || exit $?
cat $O/sum.txt
