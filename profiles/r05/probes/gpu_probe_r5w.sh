# Round 5 (for the next round's plan): the kernel at 2 waves per SIMD (512-lane blocks,
# 256 VGPRs, the CU's whole LDS for one block) against today's 4, on C4 and C5 (256 spp).
export TMPDIR=/tmp
O=gpurun_out/r05_w; mkdir -p $O
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/w2.so --config C4 C3 --steps 2 > $O/ab.txt 2>&1 || { echo "ab failed"; tail -5 $O/ab.txt; exit 1; }
timeout -k 10 900 python3 -u tools/sweep.py --lib base variants/w2.so --config C5 --spp 256 --steps 1 >> $O/ab.txt 2>&1 || { echo "ab c5 failed"; tail -5 $O/ab.txt; exit 1; }
cat $O/ab.txt
