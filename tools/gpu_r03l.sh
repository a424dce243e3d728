# One GPU call: the writer's GPU tests and throughput with 8192-member batches, and the k_huff
# phase probe.
set -o pipefail
T=${1:-r03l}
mkdir -p gpurun_out
step() {  # name, seconds, command...
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > gpurun_out/${T}_${name}.log 2>&1
  local rc=$?
  echo "step $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
A=spark-bam_amd/build/ab
step ztests 400 python -u -m pytest tests/test_zdeflate_gpu.py tests/test_deflate_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
step writer5 200 python -u tools/deflate_bench.py --mib 1024 --level 5 --exact-every 64
step hprobe 200 python -u tools/ab_inflate.py --records 4000000 --reps 1 $A/lib_hp.so
