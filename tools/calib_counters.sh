# FETCH_SIZE / WRITE_SIZE calibration on the box: each counter in its own rocprofv3 pass over
# tools/calib_counters (known byte counts in the inflate pair's access patterns), then the
# ratio per kernel.  usage: bash tools/calib_counters.sh OUTDIR
set -euo pipefail
OUT=${1:-gpurun_out/calib}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd - > /dev/null
make -s -C tools calib  # (the calibration kernels: their own target, not part of `all`)
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c -d "$OUT/$c" -o "$c" --output-format csv -- tools/calib_counters \
    > "$OUT/$c.out" 2> "$OUT/$c.log"
  cp "$(find "$OUT/$c" -name '*counter_collection.csv' -print -quit)" "$OUT/$c.csv"
done
python3 tools/calib_report.py "$OUT/FETCH_SIZE.csv" "$OUT/WRITE_SIZE.csv" "$OUT/FETCH_SIZE.out" > "$OUT/calib.json"
cat "$OUT/calib.json"
