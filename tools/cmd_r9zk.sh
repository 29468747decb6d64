# configs[3] at 1000 ZMWs under a kernel trace: when each slot's last kernel ends (the queue's tail)
mkdir -p gpurun_out/r9zk && cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
timeout -k 10 600 rocprofv3 --kernel-trace -f csv -d gpurun_out/r9zk/tr -o run -- python3 -u bench.py --workload mixed \
  --steps 1 --zmws-per-step 1000 --warmup 0 --cpu-sample 0 > gpurun_out/r9zk/mixed.json 2> gpurun_out/r9zk/mixed.err && \
python3 tools/slot_ends.py "$(find gpurun_out/r9zk/tr -name '*kernel_trace.csv' | head -1)" > gpurun_out/r9zk/slot_ends.json && \
python3 -c "import json; d=json.load(open('gpurun_out/r9zk/slot_ends.json')); print(d['ends_s'])" && \
rm -f "$(find gpurun_out/r9zk/tr -name '*kernel_trace.csv' | head -1)"
