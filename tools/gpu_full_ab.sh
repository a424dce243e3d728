# One GPU call: the full-checker parity tests, then tools/full_ab.py for in-tree and the named
# variants (spark-bam_amd/build/ab/lib_<v>.so).  usage: bash tools/gpu_full_ab.sh TAG RECORDS v1 ...
set -o pipefail
T=$1; N=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_large_offsets_gpu.py tests/test_cli.py -m gpu -x -q --timeout 300 --timeout-method thread -k "full or Full or FULL or check" > gpurun_out/${T}_fulltests.log 2>&1
echo "tests rc=$?"
timeout -k 10 200 python -u tools/full_ab.py --records $N --rtc 10 > gpurun_out/${T}_fullab.log 2>&1
for v in "$@"; do
  SBH_LIB_PATH=spark-bam_amd/build/ab/lib_$v.so timeout -k 10 200 python -u tools/full_ab.py --records $N --rtc 10 >> gpurun_out/${T}_fullab.log 2>&1
done
echo "ab rc=$?"
