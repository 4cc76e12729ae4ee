# same-box A/B of the north-star target: in-tree (one barrier) vs variants, 3 rounds
set -o pipefail
O=gpurun_out/r03o; mkdir -p $O
for r in 1 2 3; do
  for v in tree $VARIANTS; do
    lib=""; [ "$v" != tree ] && lib=variants/lib_$v.so
    IKEA_REC_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-native-side --no-eval > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
    python -c "import json;d=json.load(open('$O/$v.json'));t=d['north_star_target'];print('$r $v', d['ms_per_step'], 'target', t['frac'], t['gather_ms'], t['sampled_fwd_ms'])"
  done
done
