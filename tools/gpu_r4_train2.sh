#!/bin/bash
# round 4: a training slice of the Polar(64,32) GPU curriculum + a probe of the easy-to-hard PAC curriculum
set -e
tools/gpu_train.sh ${B1:-750} trained_crisp_64_32
tools/gpu_train.sh ${B2:-240} trained_pac_128_64_e2h
