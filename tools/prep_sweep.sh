# tile sweep for aaclip_preprocess_images (AACLIP_PREP_TILE = ty_max,tx_max,force_direct)
for cfg in 16,32,0 32,32,0 16,16,0 32,16,0 8,16,0; do
  echo "cfg $cfg"; AACLIP_PREP_TILE=$cfg timeout -k 10 60 python -u tools/kbench.py --only prep --reps 50 || exit 1
done
