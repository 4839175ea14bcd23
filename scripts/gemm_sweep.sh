#!/bin/bash
# GEMM library sweep on BERT-Large shapes; stops at the first fault/timeout.
set -u
mkdir -p gpurun_out
step() {  # step <log> <env...> -- runs micro_gemm with env
  local log=$1; shift
  env "$@" timeout -k 10 400 python scripts/micro_gemm.py > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "== $log rc=$rc"; tail -2 "gpurun_out/$log"
  if [ $rc -ge 124 ]; then echo "STOP"; exit $rc; fi
}
for v in ${SWEEP:-hipblas ck tunable}; do
  case $v in
    hipblas) step gemm_hipblas.log BLAS=hipblas ;;
    ck) step gemm_ck.log BLAS=ck ;;
    tunable) step gemm_tunable.log PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_VERBOSE=1 \
               PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_results%d.csv ;;
  esac
done
