#!/bin/bash
# kernel-trace timeline of the final-tree C2 step at one and two streams (idle, concurrency, gaps)
set -o pipefail
bash tools/prof_step.sh gpurun_out/r04_step || exit 1
grep -h "timeline\|concurr\|gap\|idle" gpurun_out/r04_step/s1.txt gpurun_out/r04_step/s2.txt
