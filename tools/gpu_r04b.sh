set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_checkers_gpu.py tests/test_blocks.py tests/test_cli.py tests/test_stream_gpu.py tests/test_gpu_parity.py tests/test_splits_gpu.py tests/test_sharded.py tests/test_records_gpu.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04b_pytest.log 2>&1
echo "tests rc=$?"
timeout -k 10 200 python -u tools/crc_bench.py --records 4000000 > gpurun_out/r04b_crc.log 2>&1 || exit 5
bash tools/gpu_round.sh fullab r04b 4000000 wc2 wc4 || exit 6
timeout -k 10 300 python -u tools/ab_inflate.py --records 400000 --reps 1 lzp > gpurun_out/r04b_lzp.log 2>&1
echo "lzp rc=$?"
