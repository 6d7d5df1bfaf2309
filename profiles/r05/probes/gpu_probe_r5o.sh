# Round 5: A2 round item sizes (A/B variants), after the final-evidence stages.
export TMPDIR=/tmp
O=gpurun_out/r05_o; mkdir -p $O
timeout -k 10 600 python3 -u tools/sweep.py --lib base variants/rcsz2.so variants/rcsz4.so variants/ripl2.so --config A2 --steps 2 > $O/a2.txt 2>&1 || { echo "a2 failed"; tail -5 $O/a2.txt; exit 1; }
cat $O/a2.txt
