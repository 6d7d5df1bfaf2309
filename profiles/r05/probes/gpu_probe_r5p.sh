# Round 5 (final code object c557a991): every reference scene at 400 px and at 1440^2, 64 spp.
export TMPDIR=/tmp
O=gpurun_out/r05_p; mkdir -p $O
S="bouncing_spheres checkered_spheres cornell_box cornell_smoke earth earth_hdr final_scene hdri mixed perlin_spheres quads simple_light triangles"
timeout -k 10 900 python3 -u tools/sweep.py --config $S --steps 3 > $O/scenes_400.txt 2>&1 || { echo "400 failed"; tail -5 $O/scenes_400.txt; exit 1; }
cat $O/scenes_400.txt
timeout -k 10 900 python3 -u tools/sweep.py --config $S --width 1440 --spp 64 --steps 2 > $O/scenes_1440.txt 2>&1 || { echo "1440 failed"; tail -5 $O/scenes_1440.txt; exit 1; }
cat $O/scenes_1440.txt
