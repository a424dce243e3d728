# One GPU call: parity (inflate/check/CLI goldens) with the op index and new CRC, CRC A/B,
# k_full A/Bs on configs B and D, the exact writer's kernel breakdown.
set -o pipefail
T=${1:-r03j}
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
step parity 300 python -u -m pytest tests/test_gpu_parity.py tests/test_cli.py -m gpu -x -q --timeout 250 --timeout-method thread
step crc 150 bash -c "for l in '' $A/lib_crcold.so; do SBH_LIB_PATH=\$l python -u tools/crc_bench.py || exit \$?; done"
step fullB 200 bash -c "for l in '' $A/lib_noix.so $A/lib_fnh.so $A/lib_nc.so; do SBH_LIB_PATH=\$l python -u tools/full_ab.py --records 4000000 --rtc 10 || exit \$?; done"
step fullD 240 bash -c "for l in '' $A/lib_noix.so; do SBH_LIB_PATH=\$l python -u tools/full_ab.py --config D --records 20000 --rtc 10 || exit \$?; done"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step wprof 200 rocprofv3 --kernel-trace --stats -d /tmp/${T}_wprof -o run -- python3 tools/deflate_bench.py --mib 256 --level 5 --reps 2
python3 tools/prof_stats.py "$(find /tmp/${T}_wprof -name '*.db' -print -quit)" > gpurun_out/${T}_writer_kernel_stats.csv
