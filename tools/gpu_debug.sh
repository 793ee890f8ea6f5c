# Targeted GPU re-runs of one test selection under the engine's A/B switches
# (each its own process and time limit; stops at the first crash / timeout).
#   gpurun -- 'bash tools/gpu_debug.sh TAG "pytest -k expr" [file]'
TAG=${1:?tag}; K=${2:?-k expression}; F=${3:-tests}
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "" "TVR_STREAM_K=0" "TVR_ROW_ATTN=0" "TVR_STREAM_K=0 TVR_ROW_ATTN=0"; do
  echo "== env: ${v:-default}" >> gpurun_out/dbg_$TAG.log
  env $v timeout -k 10 300 python -u -m pytest $F -m gpu -x -v -k "$K" --timeout 120 --timeout-method thread \
      --tb=long >> gpurun_out/dbg_$TAG.log 2>&1
  rc=$?
  echo "== rc $rc" >> gpurun_out/dbg_$TAG.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
tail -3 gpurun_out/dbg_$TAG.log
