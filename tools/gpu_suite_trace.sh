# One GPU call: the whole -m gpu suite, the default bench line, and a kernel-trace timeline of
# 8 bench steps with its device-idle gaps (tools/prof_gaps.py).  usage: bash tools/gpu_suite_trace.sh TAG
set -o pipefail
T=$1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/${T}_pytest_gpu.log 2>&1 || exit $?
echo "tests ok"
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_bench.log 2>&1 || exit $?
echo "bench ok"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/${T}_tr -o run -- python3 bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-full --no-e2e > gpurun_out/${T}_trbench.log 2>&1 || exit $?
cp "$(find /tmp/${T}_tr -name '*.db' -print -quit)" gpurun_out/${T}_trace.db
python3 tools/prof_gaps.py gpurun_out/${T}_trace.db --step-kernel k_lz --steps 6 --top 30 > gpurun_out/${T}_gaps.log 2>&1
echo "trace ok"
