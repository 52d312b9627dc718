#!/bin/bash
# round 3, call 23: prox input staging (2D chunk loads in flight at once, 3D held rows DMA'd,
# 3D monitor corners batched) -- parity, then prox times per variant
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03w
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_at_size.py -k "not c5" > $O/tests.log 2>&1
rc=$?
echo "tests rc=$rc" >> $O/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in default base nomon nodma default; do
  L=""; [ $v != default ] && L=$PWD/dev/$v/libmmadmm.so
  for wl in c4 c3; do
    MMADMM_LIB=${L:-$PWD/mm-admm_amd/lib/libmmadmm.so} WL=$wl timeout -k 10 200 python3 profiles/r02/prox_time.py >> $O/prox.jsonl 2>> $O/prox.err || exit $?
  done
done
