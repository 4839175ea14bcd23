mkdir -p gpurun_out
for cfg in "1 1" "1 0"; do set -- $cfg
  echo "== FUSED_BN=1 RESET=$1 DET=$2"
  RESET=$1 DET=$2 timeout -k 10 200 python scripts/debug/grad_repro.py 2>&1 | grep -v amdgpu.ids || exit 1
done
