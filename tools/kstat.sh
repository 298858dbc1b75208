#!/bin/bash
# usage: tools/kstat.sh file.s  -> per-kernel vgpr/sgpr/scratch/lds
awk '/\.name:/{name=$2} /\.private_segment_fixed_size:/{ps=$2} /\.sgpr_count:/{sg=$2} /\.vgpr_count:/{vg=$2; print name, "vgpr="vg, "sgpr="sg, "scratch="ps}' "$1" | sed -E 's/_ZN3npd[0-9a-z]+[0-9]+//'
