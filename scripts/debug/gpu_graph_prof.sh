mkdir -p gpurun_out
export TMPDIR=/tmp
for mode in eager graph; do
  flag=""; [ $mode = graph ] && flag="--graph"
  rm -rf /tmp/prof_$mode
  timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/prof_$mode -o run --output-format csv -- python bench.py --steps 6 --warmup 3 $flag > gpurun_out/prof_$mode.log 2>&1 || { echo "rocprof $mode failed"; exit 1; }
  f=$(find /tmp/prof_$mode -name "*kernel_trace.csv" | head -1)
  python scripts/prof_summary.py "$f" --steps 5 --title "ResNet-50 bs1024 $mode" > gpurun_out/summary_$mode.md 2>&1
done
