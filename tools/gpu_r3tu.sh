#!/bin/bash
# GPU box: tools/gpu_r3t.sh (Quiver ring / window A/B) then tools/gpu_r3u.sh (POA worker-pool A/B).
TAG=r3t bash tools/gpu_r3t.sh && TAG=r3u bash tools/gpu_r3u.sh
