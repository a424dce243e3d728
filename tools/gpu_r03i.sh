# One GPU call: the >2 GiB tests, k_full breakdown probes, the BGZF writer's throughput (exact
# level 5 and the fast coder), bench lines for configs D and E.
set -o pipefail
T=${1:-r03i}
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
step crc 150 bash -c "for l in '' $A/lib_crcold.so; do SBH_LIB_PATH=\$l python -u tools/crc_bench.py || exit \$?; done"
step large 300 python -u -m pytest tests/test_large_comp_offsets_gpu.py -m gpu -x -v --timeout 280 --timeout-method thread
step abfull 200 bash -c "for l in '' $A/lib_fo.so $A/lib_nc.so $A/lib_fnh.so; do SBH_LIB_PATH=\$l python -u tools/full_ab.py --records 4000000 --rtc 10 || exit \$?; done"
step writer5 200 python -u tools/deflate_bench.py --mib 1024 --level 5 --exact-every 64
step writerf 120 python -u tools/deflate_bench.py --mib 1024 --level -1
step benchD 240 python -u bench.py --config D --no-cpu-baseline --no-e2e
step benchE 240 python -u bench.py --config E --no-cpu-baseline --no-e2e
