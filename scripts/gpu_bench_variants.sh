#!/bin/bash
# Bench variants in one GPU session (MIOpen cache shared across steps).
set -u
mkdir -p gpurun_out
# bench.py installs the shipped MIOpen find-db / kernel cache (.miopen/) itself,
# exactly as on the driver's fresh box (scripts/miopen_db_refresh.sh rebuilds it)
run() {  # run <name> <timeout> <cmd...>
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; grep -E '^\{|\[bench\] warmup [0-9]+ steps|passed|failed|Error' "gpurun_out/$name.log" | tail -5
  if { [ $rc -ge 2 ] && [ $rc -ne 5 ]; }; then echo "STOP after $name (rc=$rc)"; exit $rc; fi
}
for v in ${VARIANTS:-default}; do
  case $v in
    tests_sel) run pytest_sel 900 python -m pytest ${TESTS_SEL:-tests} -m gpu -q ;;
    tests) run pytest_gpu 900 python -m pytest tests -m gpu -q ;;
    default) run bench_default 1200 python bench.py --steps 20 --warmup 10 ;;
    normal) MIOPEN_FIND_MODE=NORMAL run bench_normal 1200 python bench.py --steps 20 --warmup 10 ;;
    bs512) run bench_bs512 1200 python bench.py --steps 20 --warmup 10 --batch 512 ;;
    bs768) run bench_bs768 1500 python bench.py --steps 15 --warmup 8 --batch 768 ;;
    bs1024) run bench_bs1024 1500 python bench.py --steps 15 --warmup 8 --batch 1024 ;;
    bs128) run bench_bs128 1200 python bench.py --steps 20 --warmup 10 --batch 128 ;;
    bert) run bench_bert 1200 python benchmarks/bench_bert.py --steps 20 --warmup 5 ${BERT_ARGS:-} ;;
    bertprof) cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
          run rocprof_bert 1200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run --output-format csv -- python benchmarks/bench_bert.py --steps 10 --warmup 3 ${BERT_ARGS:-} ;;
    lars) run bench_lars 1200 python bench.py --steps 20 --warmup 10 --optimizer lars ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
          run rocprof 1200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 5 ${BENCH_ARGS:-} ;;
  esac
done
