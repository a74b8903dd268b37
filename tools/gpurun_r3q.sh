#!/bin/bash
# Round-3: per-block group granularity (MFHIP_SYS_GSTEP) with the placement on.
set -o pipefail
AB="MFHIP_SYS_GSTEP=8|MFHIP_SYS_GSTEP=4|MFHIP_SYS_GSTEP=2|MFHIP_SYS_GSTEP=4 MFHIP_SYS_MODEL=5000,300,186|MFHIP_SYS_GSTEP=2 MFHIP_SYS_MODEL=5000,300,186" REPS=2 bash tools/gpurun_ab.sh
CFG=ML20M AB="MFHIP_SYS_GSTEP=8|MFHIP_SYS_GSTEP=4|MFHIP_SYS_GSTEP=2" REPS=2 bash tools/gpurun_ab.sh
