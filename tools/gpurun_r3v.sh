#!/bin/bash
# Round-3: NFLX wave budget and cell model near the current defaults (placement on), A/B x3 on one box.
set -o pipefail
AB="MFHIP_SYS_WAVES=1024|MFHIP_SYS_WAVES=768|MFHIP_SYS_WAVES=768 MFHIP_SYS_MODEL=4500,300,186|MFHIP_SYS_WAVES=896" REPS=3 bash tools/gpurun_ab.sh
