set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -m gpu -x -k "head" > gpurun_out/pmc_tests.log 2>&1
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d gpurun_out/pmcA -o a -- python3 tools/headbench.py --iters 1 > gpurun_out/pmcA.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcB -o b -- python3 tools/headbench.py --iters 1 > gpurun_out/pmcB.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcC -o c -- python3 tools/headbench.py --iters 1 > gpurun_out/pmcC.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU --output-format csv -d gpurun_out/pmcD -o d -- python3 tools/headbench.py --iters 1 > gpurun_out/pmcD.log 2>&1
timeout -k 10 200 python tools/headbench.py
