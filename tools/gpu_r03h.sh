# One GPU call: the >2 GiB compressed-offset tests, k_full contig-LDS A/B, and the strong-
# scaling configs[2] line (ONE 100 GiB file on this GPU).
set -o pipefail
T=${1:-r03h}
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
step large 300 python -u -m pytest tests/test_large_comp_offsets_gpu.py -m gpu -x -v --timeout 280 --timeout-method thread
step abfull 150 bash -c "for l in '' $A/lib_c0.so; do SBH_LIB_PATH=\$l python -u tools/full_ab.py --records 4000000 --rtc 10 || exit \$?; done"
step strong 640 python -u bench.py --config C --file-gib 100 --steps 2 --warmup 1 --no-cpu-baseline
