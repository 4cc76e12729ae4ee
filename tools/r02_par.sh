cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_model_parity.py -x -v -s --timeout 300 --timeout-method thread -k top20 2>&1 | grep -E "logit bound|passed|failed|Error"
