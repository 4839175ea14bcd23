#!/bin/bash
# BERT-Large config 5 (bench_bert.py defaults: bs512, tuned GEMM table) bench + kernel profile.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python benchmarks/bench_bert.py --steps 10 --warmup 3 > gpurun_out/bert_default.log 2>&1 || exit 1
grep '"metric"' gpurun_out/bert_default.log
rm -rf /tmp/prof_bert
timeout -k 10 600 rocprofv3 --kernel-trace -d /tmp/prof_bert -o run --output-format csv -- python benchmarks/bench_bert.py --steps 5 --warmup 3 > gpurun_out/prof_bert.log 2>&1 || exit 1
f=$(find /tmp/prof_bert -name "*kernel_trace.csv" | head -1)
python scripts/prof_summary.py "$f" --steps 5 --per-step-marker adam_flat_kernel --total-steps 8 --title "BERT-Large bf16 seq128 bs512 1xMI355X (fp16 wire + Adasum path, FusedAdamW, tuned GEMM table)" > gpurun_out/summary_bert.md 2>&1
head -40 gpurun_out/summary_bert.md
