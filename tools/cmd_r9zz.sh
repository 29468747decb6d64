# device memory across repeated calls with out-of-memory reruns: current pools (ranges kept reserved) vs the pools
# before the same-VA fix (ranges freed once the next is reserved; _lib_ab)
mkdir -p gpurun_out/r9zz
for L in pbccs_amd/_lib/libpbccs_amd.so pbccs_amd/_lib_ab/libpbccs_amd.so; do
  PBCCS_LIB=$L PBCCS_DBG_VA=1 timeout -k 10 300 python3 -u -m pytest tests/test_schedule.py -k "memory_does_not_grow" -x -q --timeout 200 --timeout-method thread > gpurun_out/r9zz/p_$(basename $(dirname $L)).log 2>&1
  echo "$L: $(grep -E '^E  +AssertionError|passed|failed' gpurun_out/r9zz/p_$(basename $(dirname $L)).log | head -2 | tr '\n' ' ')"
done
