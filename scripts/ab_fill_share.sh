mkdir -p gpurun_out /tmp/m
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o /tmp/m/s70k.obj > /dev/null || exit 1
for s in 0 8 4 2; do
  echo "share=$s" 
  ERAY_FILL_SHARE=$s timeout -k 10 100 python scripts/ab_variants.py run base || exit 1
  ERAY_FILL_SHARE=$s ERAY_AB_MESH=/tmp/m/s70k.obj timeout -k 10 100 python scripts/ab_variants.py run base || exit 1
  ERAY_FILL_SHARE=$s ERAY_AB_MESH=/tmp/m/s70k.obj ERAY_AB_W=3840 ERAY_AB_H=2160 timeout -k 10 100 python scripts/ab_variants.py run base || exit 1
done
