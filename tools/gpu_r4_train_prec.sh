#!/bin/bash
# round 4: a training slice of both GPU curricula, then the GRU precision study on the current Polar(64,32) fixture
set -e
tools/gpu_train.sh ${B1:-650} trained_crisp_64_32
tools/gpu_train.sh ${B2:-300} trained_pac_128_64
timeout -k 10 300 python -u tools/gru_precision.py --n 65536 --out gpurun_out/gru_precision.json > gpurun_out/gru_precision.log 2>&1
