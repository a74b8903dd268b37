#!/bin/bash
# Round-3: ML20M group model with cheaper single-run pairs (k=64 single-run cells run 126-177 ns per
# pair in situ, the model's 186 ns makes the hot-item block's G too small).
set -o pipefail
CFG=ML20M AB="MFHIP_SYS_MODEL=6000,300,186|MFHIP_SYS_MODEL=6000,300,150|MFHIP_SYS_MODEL=6000,300,130|MFHIP_SYS_MODEL=6000,300,110|MFHIP_SYS_MODEL=6000,300,130 MFHIP_SYS_GSTEP=4" REPS=2 bash tools/gpurun_ab.sh
