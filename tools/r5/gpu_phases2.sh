#!/bin/bash
# round 5: per-phase cycles of the step kernel from the MJL_TIMING build (tools/phase_times.py), final sources
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5p
mkdir -p $O
MJX355_LIB=$PWD/mujoco-mjx-lab_amd/mjx_amd/libmjx355_timing.so timeout -k 10 300 python tools/phase_times.py > $O/phases.txt 2>&1 \
  || { tail -20 $O/phases.txt; exit 1; }
cat $O/phases.txt
