set -o pipefail
bash profiles/collect.sh gpurun_out/p_c3 "--workload c3 --steps 4 --warmup 1 --no-cpu-baseline --no-expansion --no-ingest --no-latency" sdh_part_spec || exit 1
python3 profiles/summarize.py gpurun_out/p_c3 gpurun_out/r5_c3 sdh_part_spec c3 1000 1048576 > gpurun_out/p_c3.sum || exit 1
