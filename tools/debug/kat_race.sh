cd $GRAFT_REPO_ROOT
for e in "GPU_MAX_HW_QUEUES=4" "GPU_MAX_HW_QUEUES=16" "GPU_MAX_HW_QUEUES=16 AMD_SERIALIZE_KERNEL=3" "GPU_MAX_HW_QUEUES=16 AMD_SERIALIZE_COPY=3"; do
  echo "=== $e"
  env $e timeout -k 5 60 python -u tools/debug/kat_race.py > gpurun_out/dbg_$(echo $e | tr ' =' '__').log 2>&1 || { echo FAIL; exit 1; }
  grep BAD gpurun_out/dbg_$(echo $e | tr ' =' '__').log
done
