#!/bin/bash
# Round-3: the cross-cell record preload (PRE) re-measured with the placement on, per config.
set -o pipefail
CFG=ML20M AB="MFHIP_CELL_PRELOAD=0|MFHIP_CELL_PRELOAD=1" REPS=2 bash tools/gpurun_ab.sh
CFG=NFLX AB="MFHIP_CELL_PRELOAD=1|MFHIP_CELL_PRELOAD=0" REPS=2 bash tools/gpurun_ab.sh
