# final pass A: the ratchet-touching tests, then the C2 / C3 / C4 profiles
set -o pipefail
bash tools/r5_rec4c.sh || exit 1
bash tools/r5_prof.sh c2 c3 c4 || exit 1
