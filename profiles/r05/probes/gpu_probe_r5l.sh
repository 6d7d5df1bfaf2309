# Round 5: small frames wholly in 4-sample chunks (default), claims of up to 128 items for the
# rounds' few-sample items, claim size per wave share (A/B variants).
export TMPDIR=/tmp
O=gpurun_out/r05_l; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py tests/test_gpu_adaptive.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "GPU TESTS FAILED"; tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 600 python3 -u tools/sweep.py --lib base variants/claim4.so variants/claim2.so --config C1 --steps 30 > $O/c1.txt 2>&1 || { echo "c1 failed"; tail -5 $O/c1.txt; exit 1; }
timeout -k 10 600 python3 -u tools/sweep.py --lib base variants/claim4.so variants/claim2.so --config C1 --steps 30 >> $O/c1.txt 2>&1 || { echo "c1 failed"; tail -5 $O/c1.txt; exit 1; }
cat $O/c1.txt
timeout -k 10 600 python3 -u tools/sweep.py --lib base variants/claim4.so variants/claim2.so --config A2 A1 --steps 2 > $O/adaptive.txt 2>&1 || { echo "adaptive failed"; tail -5 $O/adaptive.txt; exit 1; }
cat $O/adaptive.txt
timeout -k 10 300 python3 -u tools/sweep.py --config final_scene --steps 3 > $O/fs400.txt 2>&1 || { echo "fs400 failed"; tail -5 $O/fs400.txt; exit 1; }
timeout -k 10 300 python3 -u tools/sweep.py --config final_scene --steps 3 --fine-chunk 1 --tail-pct 200 >> $O/fs400.txt 2>&1 || { echo "fs400 failed"; tail -5 $O/fs400.txt; exit 1; }
cat $O/fs400.txt
timeout -k 10 600 python3 -u tools/sweep.py --lib base variants/claim4.so --config C2 C4 --steps 2 > $O/big.txt 2>&1 || { echo "big failed"; tail -5 $O/big.txt; exit 1; }
cat $O/big.txt
