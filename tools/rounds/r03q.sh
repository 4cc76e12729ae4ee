set -o pipefail
O=gpurun_out/r03q; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 python $R/tools/sampbench.py --HF 128 --prec f32x6 --fused --planes > $R/$O/cold.txt 2>&1
timeout -k 10 120 python $R/tools/sampbench.py --HF 128 --prec f32x6 --fused --planes --hot > $R/$O/hot.txt 2>&1
timeout -k 10 120 python $R/tools/sampbench.py --HF 128 --prec f32x6 --fused --planes --A 8192 > $R/$O/small.txt 2>&1
cat $R/$O/*.txt
