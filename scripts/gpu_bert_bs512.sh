set -u; mkdir -p gpurun_out
timeout -k 10 300 python benchmarks/bench_bert.py > gpurun_out/bert256.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/bert256.log
timeout -k 10 300 python benchmarks/bench_bert.py --batch 512 > gpurun_out/bert512.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/bert512.log
cp .tunableop/bert_large_bs256_seq128.csv gpurun_out/bert_large_bs512_seq128.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/bert_large_bs512_seq128.csv \
  timeout -k 10 700 python benchmarks/bench_bert.py --batch 512 --steps 5 --warmup 3 > gpurun_out/bert512_tune.log 2>&1 || exit 1
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/bert_large_bs512_seq128.csv \
  timeout -k 10 300 python benchmarks/bench_bert.py --batch 512 > gpurun_out/bert512_tuned.log 2>&1 || exit 1
grep -o '"value": [0-9.]*' gpurun_out/bert512_tuned.log
