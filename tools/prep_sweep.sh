# sweep for aaclip_preprocess_images: two-pass rows per horizontal workgroup (AACLIP_PREP_HROWS)
# and the single-kernel tile path (AACLIP_PREP_TILE = ty_max,tx_max,force_direct)
for r in 2 4 8 16; do
  echo "hrows $r"; AACLIP_PREP_HROWS=$r timeout -k 10 60 python -u tools/kbench.py --only prep --reps 50 || exit 1
done
echo "single 16,32"; AACLIP_PREP_TILE=16,32,0 timeout -k 10 60 python -u tools/kbench.py --only prep --reps 50 || exit 1
