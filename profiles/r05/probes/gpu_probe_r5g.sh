export TMPDIR=/tmp
O=gpurun_out/r05_g; mkdir -p $O
timeout -k 10 600 python3 -u tools/sweep.py --lib base variants/newsites.so variants/reuse.so --config final_scene --width 1440 --spp 64 --steps 2 --leaf-batch 24 48 > $O/fs_ab.txt 2>&1 || { echo "fs ab failed"; tail -5 $O/fs_ab.txt; exit 1; }
cat $O/fs_ab.txt
timeout -k 10 300 python3 -u tools/sweep.py --config C4 --steps 2 --leaf-batch 10 12 14 > $O/c4.txt 2>&1 || { echo "c4 failed"; tail -5 $O/c4.txt; exit 1; }
cat $O/c4.txt
for spec in "final_scene --width 1440 --spp 64" "C4"; do
  set -- $spec
  GS_LIB=$PWD/grayshift_amd/variants/stamps.so timeout -k 10 300 python3 tools/stamps.py --config $spec > $O/stamps_$1.txt 2> $O/stamps_$1.err || { echo "stamps $1 failed"; tail -5 $O/stamps_$1.err; exit 1; }
  echo "== stamps $1"; cat $O/stamps_$1.txt
done
bash tools/gpu_probe_c1.sh
