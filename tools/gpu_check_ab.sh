# One GPU call: the whole -m gpu suite, then the in-tree inflate A/B line (4 M records, config B)
# and the default bench line.  usage: bash tools/gpu_check_ab.sh TAG
set -o pipefail
T=$1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || exit $?
echo "tests ok"
timeout -k 10 300 python -u tools/ab_inflate.py --records 4000000 > gpurun_out/${T}_ab.log 2>&1 || exit $?
echo "ab ok"
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || exit $?
echo "bench ok"
