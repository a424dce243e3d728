#!/bin/bash
# rocprofv3 counter passes over a short bench run (one pass per counter group: rocprofv3 does
# not split groups over passes; at most 8 SQ / 4 TCC counters per pass on gfx950), then the
# per-kernel summaries.  Usage (on the GPU box, from the repo root):
#   bash tools/pmc_collect.sh gpurun_out/pmc "--no-cpu-baseline --no-e2e --steps 2 --warmup 1"
set -euo pipefail
OUT=${1:-gpurun_out/pmc}
ARGS=${2:---no-cpu-baseline --no-e2e --no-facade --steps 2 --warmup 1}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd - > /dev/null
pass() {  # name, counters...
  local name=$1
  shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d "$OUT/$name" -o "$name" --output-format csv -- \
    python3 bench.py $ARGS > "$OUT/$name.bench.json" 2> "$OUT/$name.log"
  local f
  f=$(find "$OUT/$name" -name "*counter_collection.csv" -print -quit)
  cp "$f" "$OUT/$name.csv"
  echo "pass $name done"
}
pass sq_lds SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS
pass sq_wait SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES
pass fetch FETCH_SIZE
pass write WRITE_SIZE
python3 -c "import bench; print(bench.kernel_src_hash())" > "$OUT/src_hash"
python3 tools/pmc_summary.py "$OUT/sq_lds.csv" > "$OUT/sq_lds.txt"
python3 tools/pmc_summary.py "$OUT/sq_wait.csv" > "$OUT/sq_wait.txt"
python3 tools/pmc_traffic.py "$OUT/fetch.csv" "$OUT/write.csv" > "$OUT/traffic.json"
python3 tools/pmc_derived.py "$OUT" > "$OUT/derived.json"
echo "pmc ok"
