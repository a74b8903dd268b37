#!/bin/bash
# Round-3: NFLX wave budgets between 512 (every CU <= 2 waves) and the model's own 647.
set -o pipefail
AB="MFHIP_SYS_WAVES=1024|MFHIP_SYS_WAVES=600|MFHIP_SYS_WAVES=560" REPS=2 bash tools/gpurun_ab.sh
