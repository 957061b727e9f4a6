mkdir -p gpurun_out/r6e
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_metrics.py tests/test_spec_view.py tests/test_dropin.py tests/test_abi.py > gpurun_out/r6e/t.log 2>&1
