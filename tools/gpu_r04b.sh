set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_checkers_gpu.py tests/test_blocks.py tests/test_cli.py tests/test_stream_gpu.py tests/test_gpu_parity.py tests/test_splits_gpu.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04b_pytest.log 2>&1
