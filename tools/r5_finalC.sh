# final pass C: the C5 profile and the C5 line
set -o pipefail
bash tools/r5_prof.sh c5 || exit 1
timeout -k 10 700 python -u bench.py --workload c5 > gpurun_out/line_c5.log 2> gpurun_out/line_c5.err || { tail -20 gpurun_out/line_c5.err; exit 1; }
tail -1 gpurun_out/line_c5.log | cut -c1-200
