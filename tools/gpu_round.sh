# One GPU call, by mode (on the box, from the repo root; everything lands in gpurun_out/TAG_*).
# Every GPU step has its own time limit and the steps are chained: the first failure ends the call.
#
#   bash tools/gpu_round.sh round TAG              -m gpu suite, bench (config B), its rocprofv3 kernel
#                                                  summary, bench lines for configs D and E
#   bash tools/gpu_round.sh tests TAG FILE...      the -m gpu tests of the named files, verbose
#   bash tools/gpu_round.sh bench TAG ARGS...      one bench.py line with ARGS
#   bash tools/gpu_round.sh prof TAG ARGS...       rocprofv3 --kernel-trace --stats of bench.py ARGS
#   bash tools/gpu_round.sh ab TAG CONFIG RECORDS V...   inflate A/B: in-tree vs spark-bam_amd/build/ab/lib_V.so
#   bash tools/gpu_round.sh fullab TAG RECORDS V...      full-checker A/B (tools/full_ab.py), same variants
#   bash tools/gpu_round.sh pmc TAG ARGS...        counter passes (tools/pmc_collect.sh) over bench.py ARGS
#   bash tools/gpu_round.sh trace TAG              kernel-trace timeline of 8 bench steps + idle gaps
#   bash tools/gpu_round.sh ftrace TAG LASTMS ARGS...  kernel-trace of bench.py ARGS, idle gaps of its last LASTMS ms
#   bash tools/gpu_round.sh abenv TAG "ENV_A" "ENV_B" ARGS...  bench.py ABAB of an environment toggle
#   bash tools/gpu_round.sh allpos TAG GIB ARGS...  check-bam -s over configs[2]'s one GIB-GiB file
#                                                  (tools/allpos_configC.py: a 2 GiB rehearsal first)
set -o pipefail
M=$1; T=$2; shift 2
mkdir -p gpurun_out
PYT="python -u -m pytest -m gpu --timeout 300 --timeout-method thread"
prof_env() { cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; }
case "$M" in
round)
  timeout -k 10 900 $PYT tests -x -q > gpurun_out/${T}_pytest_gpu.log 2>&1 || exit 1
  timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 2
  prof_env
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/${T}_bprof -o run -- python3 bench.py --steps 5 --warmup 2 \
    --no-cpu-baseline --no-full --no-e2e --no-facade > gpurun_out/${T}_bprof.json 2> gpurun_out/${T}_bprof.log || exit 3
  python3 tools/prof_stats.py "$(find /tmp/${T}_bprof -name '*.db' -print -quit)" > gpurun_out/${T}_kernel_stats.csv || exit 3
  timeout -k 10 300 python -u bench.py --config D --no-cpu-baseline --no-full --no-e2e --no-facade > gpurun_out/${T}_benchD.json \
    2> gpurun_out/${T}_benchD.err || exit 4
  timeout -k 10 300 python -u bench.py --config E --no-cpu-baseline --no-full --no-e2e --no-facade > gpurun_out/${T}_benchE.json \
    2> gpurun_out/${T}_benchE.err || exit 5
  ;;
tests)
  timeout -k 10 1000 $PYT "$@" -v > gpurun_out/${T}_pytest.log 2>&1 || exit 1
  ;;
bench)
  timeout -k 10 600 python -u bench.py "$@" > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 2
  ;;
prof)
  prof_env
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/${T}_prof -o run -- python3 bench.py "$@" \
    > gpurun_out/${T}_prof.json 2> gpurun_out/${T}_prof.log || exit 3
  python3 tools/prof_stats.py "$(find /tmp/${T}_prof -name '*.db' -print -quit)" > gpurun_out/${T}_kernel_stats.csv || exit 3
  ;;
ab)
  C=$1; N=$2; shift 2
  L=""
  for v in "$@"; do L="$L spark-bam_amd/build/ab/lib_$v.so"; done
  timeout -k 10 900 python -u tools/ab_inflate.py --config $C --records $N --rounds ${AB_ROUNDS:-1} $L > gpurun_out/${T}_ab$C.log 2>&1 || exit 6
  ;;
fullab)
  N=$1; shift
  timeout -k 10 200 python -u tools/full_ab.py --records $N --rtc 10 > gpurun_out/${T}_fullab.log 2>&1 || exit 7
  for v in "$@"; do
    SBH_LIB_PATH=spark-bam_amd/build/ab/lib_$v.so timeout -k 10 200 python -u tools/full_ab.py --records $N --rtc 10 \
      >> gpurun_out/${T}_fullab.log 2>&1 || exit 7
  done
  ;;
pmc)
  bash tools/pmc_collect.sh gpurun_out/${T}_pmc "$*" > gpurun_out/${T}_pmc.log 2>&1 || exit 8
  ;;
trace)
  prof_env
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/${T}_tr -o run -- python3 bench.py --steps 8 --warmup 2 \
    --no-cpu-baseline --no-full --no-e2e > gpurun_out/${T}_trbench.log 2>&1 || exit 9
  cp "$(find /tmp/${T}_tr -name '*.db' -print -quit)" gpurun_out/${T}_trace.db
  python3 tools/prof_gaps.py gpurun_out/${T}_trace.db --step-kernel k_lz --steps 6 --top 30 > gpurun_out/${T}_gaps.log 2>&1
  ;;
ftrace)
  # kernel-trace timeline of bench.py ARGS and the busy / idle split of its last LASTMS ms
  L=$1; shift
  prof_env
  timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/${T}_ft -o run -- python3 bench.py "$@" \
    > gpurun_out/${T}_ftrace.json 2> gpurun_out/${T}_ftrace.err || exit 12
  cp "$(find /tmp/${T}_ft -name '*.db' -print -quit)" gpurun_out/${T}_ftrace.db
  python3 tools/prof_gaps.py gpurun_out/${T}_ftrace.db --last-ms $L --top 30 > gpurun_out/${T}_fgaps.log 2>&1
  ;;
abenv)
  # bench.py A/B of an environment toggle: abenv TAG "ENV_A" "ENV_B" ARGS...
  timeout -k 10 1500 bash tools/ab_env.sh "$T" "$@" || exit 13
  ;;
allpos)
  G=$1; shift
  timeout -k 10 300 python -u tools/allpos_configC.py --file-gib 2 "$@" > gpurun_out/${T}_allpos2.log 2>&1 || exit 10
  timeout -k 10 1000 python -u tools/allpos_configC.py --file-gib $G "$@" > gpurun_out/${T}_allpos.log 2>&1 || exit 11
  ;;
*)
  echo "unknown mode $M" >&2
  exit 64
  ;;
esac
echo "$M ok"
