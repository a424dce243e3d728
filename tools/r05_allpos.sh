# check-bam -s over configs[2]-shaped files streamed through HBM (sbh_check_stream): the GPU
# tests of the streamed paths, a 4 GiB timing with its kernel trace, then (optional) the
# full-size file.  usage: bash tools/r05_allpos.sh TAG [GIB] [--full]
set -o pipefail
T=$1; G=${2:-0}; shift 2 2>/dev/null; X="$*"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu --timeout 300 --timeout-method thread -x -q tests/test_stream_gpu.py \
  tests/test_cli.py tests/test_splits_gpu.py > gpurun_out/${T}_pytest.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/allpos_configC.py --file-gib 4 $X > gpurun_out/${T}_allpos4.log 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d /tmp/${T}_p -o run -- python3 tools/allpos_configC.py --file-gib 4 $X \
  > gpurun_out/${T}_allpos4_prof.log 2>&1 || exit 3
DB=$(find /tmp/${T}_p -name '*.db' -print -quit)
python3 tools/prof_stats.py "$DB" > gpurun_out/${T}_kstats.csv || exit 4
python3 tools/prof_gaps.py "$DB" --step-kernel k_lz --steps 3 --top 25 > gpurun_out/${T}_gaps.log 2>&1
if [ "$G" != "0" ]; then
  timeout -k 10 1000 python3 -u tools/allpos_configC.py --file-gib $G $X > gpurun_out/${T}_allpos${G}.log 2>&1 || exit 5
fi
echo done
