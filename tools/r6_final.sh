# the round's final measurements at the final tree: PMC profiles of the workloads whose kernel sources
# changed since profiles/r6_* (copied into profiles/ on the box so the lines find them), then every line
set -o pipefail
bash tools/prof.sh r6 $* || exit 1
for w in $*; do rm -rf profiles/r6_$w && cp -r gpurun_out/r6_$w profiles/r6_$w || exit 1; done
bash tools/lines.sh c5
