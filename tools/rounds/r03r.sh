set -o pipefail
O=gpurun_out/r03r; mkdir -p $O
R=$GRAFT_REPO_ROOT
for v in "" variants/lib_pf.so variants/lib_pf0.so "" variants/lib_pf.so variants/lib_pf0.so; do
  IKEA_REC_HIP_LIB=$v timeout -k 10 120 python tools/sampbench.py --HF 128 --prec f32x6 --fused --planes 2>&1 | grep fused | sed "s|^|lib=${v:-tree} |" || exit 1
done
