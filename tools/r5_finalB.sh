# final pass B: the C5 profile, then the C2 / C3 / C4 lines
set -o pipefail
bash tools/r5_prof.sh c5 || exit 1
bash tools/lines.sh || exit 1
