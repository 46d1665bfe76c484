#!/bin/bash
# final profiles at HEAD: C2 (headline), C3, C4
set -o pipefail
bash tools/r3_prof.sh c2 c3 c4
