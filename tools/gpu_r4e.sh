#!/bin/bash
# Round 4: confirm the stamps-hang cause (wait-only vs bound-only probe builds on the media
# scenes), then the fixed stamps build's phase split of final_scene, cornell_smoke and C4.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4e
mkdir -p $O
for v in st_wait_unb st_nowait_b stamps; do
  for sc in cornell_smoke final_scene; do
    GS_LIB=$R/grayshift_amd/variants/$v.so timeout -k 5 45 python3 -u $R/tools/stamps.py --config $sc --width 96 --spp 4 > $O/probe_${v}_$sc.txt 2>&1
    echo "probe $v $sc rc=$?"; grep -v amdgpu.ids $O/probe_${v}_$sc.txt | head -3
  done
done
for spec in "final_scene 1440 64" "cornell_smoke 1440 64" "C4 1920 512"; do
  set -- $spec
  GS_LIB=$R/grayshift_amd/variants/stamps.so timeout -k 10 150 python3 $R/tools/stamps.py --config $1 --width $2 --spp $3 > $O/stamps_$1.txt 2> $O/stamps_$1.err || { echo "stamps $1 failed rc=$?"; tail -3 $O/stamps_$1.err; exit 1; }
  echo "== stamps $1"; cat $O/stamps_$1.txt
done
