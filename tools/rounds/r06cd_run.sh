#!/bin/bash
# Round 6: r06c (copy roof, transform sizes, ladder) then r06d (message forms at every small size, long mix).
set -o pipefail
bash tools/rounds/r06d_run.sh && bash tools/rounds/r06c_run.sh
